/*
 * aimx_h5.h — C ABI of the HDF5 molecule stream (libaimx_h5.so, host C++, links the HDF5 C
 * library). It reads and writes the reference's precomputed-dataset format:
 *   writer  src/datasets/features.py:381-431, 537-596 (precompute_and_write_hdf5_parallel_chunked)
 *   reader  src/datasets/molecular.py:102-329 (HDF5MolecularIterableDataset)
 * /data is a 1-D vlen-uint8 dataset of pickled record dicts, /index_map int32, /metadata a group
 * of attributes. Records are decoded without executing anything (host/pickle_lite.h) into a
 * molecule store of include/aimx_host.h, which the native collator turns into batches.
 * Functions return 0 on success, negative codes on error (AIMX_HOST_* of aimx_host.h, plus the
 * two below); no function raises, prints or aborts.
 */
#ifndef AIMX_H5_H_
#define AIMX_H5_H_

#include <stddef.h>
#include <stdint.h>

#include "aimx_host.h"

#ifdef __cplusplus
extern "C" {
#endif

#define AIMX_H5_EIO (-10)     /* the HDF5 library failed to open / read / write the file */
#define AIMX_H5_EFORMAT (-11) /* not the reference layout (no 1-D vlen /data, bad index_map) */

typedef struct AimxH5Info {
  int64_t n_records;             /* length of /data */
  int64_t num_samples;           /* metadata attr (n_records when absent) */
  int64_t max_hops;              /* metadata attr (-1 when absent) */
  int32_t preprocessing_applied; /* metadata attr, else metadata/sae attr 'applied' (molecular.py:159-174) */
  char task_type[32];            /* metadata attr ("" when absent) */
  int32_t direct_read;           /* reader: 1 = records come straight from the memory-mapped file
                                    (contiguous /data, checked against H5Dread at open), 0 = H5Dread */
} AimxH5Info;

typedef struct aimx_h5_reader aimx_h5_reader;
typedef struct aimx_h5_writer aimx_h5_writer;

/* Open for reading; loads /index_map (identity when absent, as molecular.py:138-142). */
int aimx_h5_open(const char* path, aimx_h5_reader** out);
/* Test hook: allow (1, default) or forbid (0) the direct memory-mapped record path in later
 * aimx_h5_open calls (AimxH5Info.direct_read), so both read paths can be compared. */
void aimx_h5_set_direct(int32_t allow);
void aimx_h5_close(aimx_h5_reader* r);
int aimx_h5_info(const aimx_h5_reader* r, AimxH5Info* out);

/* Read records index_map[pos[k]] (k < n, request order; one hyperslab read when they are
 * consecutive, a point selection otherwise), decode them on n_threads threads and return a store
 * with their atom features (atom_type, hydrogen_count, degree, hybridization), the first n_hops
 * hop arrays, n_tasks targets and total charge. As the reference's _build_data_object
 * (molecular.py:253-329) skips None records, invalid records are skipped: *n_valid molecules are
 * stored, and valid_pos (nullable, capacity n) receives the pos value of each stored molecule. */
int aimx_h5_read_store(aimx_h5_reader* r, const int64_t* pos, int64_t n, int32_t n_hops, int32_t n_tasks,
                       int32_t n_threads, aimx_mol_store** out, int64_t* n_valid, int64_t* valid_pos);

/* Writer: the file features.py:416-431 creates — /data (n_records vlen uint8), /index_map
 * (identity), /metadata attrs num_samples, task_type, max_hops, preprocessing_applied, group sae
 * (applied, note) — with h5py's type mapping (int64 attrs, bool as an int8 FALSE/TRUE enum,
 * str as variable-length UTF-8). put() writes records [start, start+count): record k is
 * bytes[offsets[k] .. offsets[k+1]). close() adds metadata attr estimated_valid_pct. */
int aimx_h5_writer_create(const char* path, int64_t n_records, const AimxH5Info* meta, aimx_h5_writer** out);
int aimx_h5_writer_put(aimx_h5_writer* w, int64_t start, int64_t count, const uint8_t* bytes,
                       const int64_t* offsets);
int aimx_h5_writer_close(aimx_h5_writer* w, double estimated_valid_pct);

/* Decode one record (a pickled dict) without a file: 1 = valid (n_atoms, n_pairs set), 0 = a
 * record the reader would skip, negative = bad arguments. */
int32_t aimx_h5_decode_record(const uint8_t* bytes, int64_t n, int32_t n_hops, int32_t n_tasks, int32_t* n_atoms,
                              int64_t* n_pairs);

#ifdef __cplusplus
}
#endif

#endif /* AIMX_H5_H_ */
