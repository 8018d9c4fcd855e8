/*
 * aimx_host.h — C ABI of the native (host, C++) batch builder that feeds the MI355X hot path.
 *
 * Library: aimnet-x2d_amd/lib/libaimx_host.so (g++, no GPU code; loads and runs on any host).
 * It replaces the two reference host stages that produce the hot path's inputs:
 *   * multi-hop BFS pair lists — src/datasets/features.py:82-150
 *     (build_numba_adjacency_list + compute_multi_hop_edges_bfs_numba);
 *   * collate — src/datasets/molecular.py:339-458 (MyBatch.from_data_list): per-molecule hop
 *     pairs offset by the molecule's atom offset only, molecule-major then hop-major, transposed
 *     to multi_hop_edge_indices [E, 2] int64; batch_indices = repeat_interleave(arange(G), atoms).
 * Outputs are bit-identical to the reference (tests/test_host_collate.py vs tests/golden/edges.npz
 * and vs aimx.data). Output buffers are owned by the caller (typically one pinned host blob that
 * is DMA'd to HBM with a single async copy, aimx/feed.py). Functions return 0 (AIMX_OK) on
 * success and a negative code on error; no function raises or aborts.
 *
 * Threading: a collator owns a persistent worker pool; calls on one collator must not overlap,
 * separate collators are independent. A store is immutable after creation and may be shared.
 */
#ifndef AIMX_HOST_H_
#define AIMX_HOST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AIMX_HOST_OK 0
#define AIMX_HOST_EARG (-1)      /* invalid argument (null pointer, negative size, bad index) */
#define AIMX_HOST_ESPACE (-2)    /* caller capacity too small (padded fill: n_max / e_max) */
#define AIMX_HOST_ENOMEM (-3)    /* host allocation failed */
#define AIMX_HOST_ESTATE (-4)    /* write without a matching plan */

/* Library identity: "aimx_host/<version>". */
const char* aimx_host_version(void);

/* ------------------------------------------------------------------------------------------
 * Single-molecule BFS (reference features.py:97-150; the adjacency is the reference's
 * `adj_matrix > 0` with self-loops skipped, features.py:82-95, built here from a bond list).
 *   bonds: int32 [n_bonds, 2] local atom indices (either orientation, duplicates allowed)
 *   pairs: int32 [cap, 2] output (u, w) rows, hop-major; hop_counts[max_hops] pairs per hop
 * Returns the total number of pairs (>= 0); if it exceeds `cap`, nothing beyond cap is written
 * and the caller retries with a larger buffer. Negative on invalid input.
 * ------------------------------------------------------------------------------------------ */
int64_t aimx_bfs_multi_hop(int32_t n_atoms, const int32_t* bonds, int64_t n_bonds, int32_t max_hops,
                           int32_t* pairs, int64_t cap, int64_t* hop_counts);

/* ------------------------------------------------------------------------------------------
 * Molecule store: the dataset's per-molecule records (the fields of one reference Data object
 * that collate reads: x / atom_features_map, multi_hop_edges via the bonds, target,
 * total_charge; molecular.py:345-458). Arrays are copied in.
 *   atom_ptr[n_mols+1], bond_ptr[n_mols+1]: offsets into feats rows / bonds rows
 *   bonds int32 [bond_ptr[n_mols], 2] local indices; feats int32 [atom_ptr[n_mols], n_feat]
 *   targets f32 [n_mols, n_tasks] (NULL: zeros), total_charge f32 [n_mols] (NULL: zeros)
 * precompute_hops > 0 caches every molecule's hop pairs for that many hops at creation (as the
 * reference stores multi_hop_edges in its dataset, features.py:416-431); otherwise the BFS runs
 * inside every collate (streaming datasets).
 * ------------------------------------------------------------------------------------------ */
typedef struct aimx_mol_store aimx_mol_store;

int aimx_store_create(int64_t n_mols, const int64_t* atom_ptr, const int64_t* bond_ptr,
                      const int32_t* bonds, const int32_t* feats, int32_t n_feat,
                      const float* targets, int32_t n_tasks, const float* total_charge,
                      int32_t precompute_hops, int32_t n_threads, aimx_mol_store** out);
/* A store from precomputed hop pair lists (the reference's stored multi_hop_edges,
 * features.py:318-334 / molecular.py:307-309, e.g. decoded from an HDF5 stream by
 * libaimx_h5.so): molecule m's hop h pairs are pairs[hop_ptr[m*n_hops+h] .. hop_ptr[m*n_hops+h+1])
 * as (u, w) rows of local atom indices, in the reference's stored order. hop_ptr has
 * n_mols*n_hops+1 entries starting at 0; collate with the same max_hops = n_hops. */
int aimx_store_create_hops(int64_t n_mols, const int64_t* atom_ptr, const int32_t* feats, int32_t n_feat,
                           int32_t n_hops, const int64_t* hop_ptr, const int32_t* pairs, const float* targets,
                           int32_t n_tasks, const float* total_charge, aimx_mol_store** out);
void aimx_store_destroy(aimx_mol_store* store);
int64_t aimx_store_num_molecules(const aimx_mol_store* store);
int64_t aimx_store_num_atoms(const aimx_mol_store* store, int64_t mol);
/* Atom counts of every molecule at once: out[n_mols] (one call instead of n_mols). */
int aimx_store_atom_counts(const aimx_mol_store* store, int64_t* out);

/* ------------------------------------------------------------------------------------------
 * Collator: plan (BFS or cache lookup for the G molecules of a batch, sizes) then write into
 * caller buffers. Reference MyBatch.from_data_list (molecular.py:339-458) for the real part and
 * SURVEY.md §8d "padded batches" for the static-shape padding used by HIP-graph replay.
 * ------------------------------------------------------------------------------------------ */
typedef struct aimx_collator aimx_collator;

typedef struct AimxCollateOut {
  int64_t* feat[8];       /* n_feat columns, each int64 [n_rows] (reference atom_features_map) */
  int64_t* edges;         /* int64 [e_rows, 2]: (row 0, row 1) of the hop arrays + atom offset */
  int64_t* batch;         /* int64 [n_rows] molecule id per atom */
  float* total_charges;   /* f32 [g_rows] (NULL: skipped) */
  float* targets;         /* f32 [g_rows, n_tasks] (NULL: skipped) */
  int64_t* n_atoms;       /* int64 [g_rows] atoms per molecule (NULL: skipped) */
  /* static padding (n_max == 0: no padding, rows = the real sizes). Otherwise n_max > N,
   * e_max >= E, pad_mols >= 1: slack atoms form pad_mols molecules G..G+pad_mols-1 (sizes as
   * equal as possible), slack edges are self-pairs spread over the padding atoms. */
  int64_t n_max, e_max;
  int32_t pad_mols;
} AimxCollateOut;

int aimx_collator_create(int32_t max_hops, int32_t n_threads, aimx_collator** out);
void aimx_collator_destroy(aimx_collator* c);
/* Plan a batch: idx[G] molecule ids into `store`; returns N (atoms) and E (pairs). */
int aimx_collate_plan(aimx_collator* c, const aimx_mol_store* store, const int64_t* idx, int64_t G,
                      int64_t* n_atoms, int64_t* n_edges);
/* Write the planned batch (same store; the plan stays valid until the next plan). */
int aimx_collate_write(aimx_collator* c, const AimxCollateOut* out);

/* ------------------------------------------------------------------------------------------
 * Host-built CSR views of a collated batch: the same three stable CSRs the device builder
 * aimx_csr_build_multi (include/aimx.h) makes at the start of every forward, computed here by the
 * batch builder and shipped inside the batch blob, so a train step starts with its CSRs already
 * in HBM (no per-step count / scan / fill / order launches).
 *   edges int64 [E, 2] (column 0 target, column 1 source: multi_hop_edge_indices), batch int64 [N]
 *   fwd:   rows hops*N keyed by target,  col = source mod N (Python-style), fwd_rowptr[hops*N+1]
 *   bwd:   rows N keyed by source mod N, col = target,                      bwd_rowptr[N+1]
 *   graph: rows G keyed by batch[i],     col = i,                           graph_rowptr[G+1]
 * Items keep ascending order inside a row (the reference's summation order). Returns AIMX_HOST_EARG
 * when a target is outside [0, hops*N), a batch index outside [0, G), or N == 0 with E > 0 (the
 * device builder's status word cases), and for E, N, G, hops sizes that do not fit int32 CSRs.
 * ------------------------------------------------------------------------------------------ */
int aimx_csr_host_build(const int64_t* edges, int64_t E, const int64_t* batch, int64_t N, int64_t G, int32_t hops,
                        int32_t* fwd_rowptr, int32_t* fwd_col, int32_t* bwd_rowptr, int32_t* bwd_col,
                        int32_t* graph_rowptr, int32_t* graph_col);

/* aimx_csr_host_build's contract and bit-identical output, built by the collator's worker pool
 * for the batch it has just written (aimx_collate_write into these edges / batch buffers, padded
 * or not): each molecule's edges join only its own atoms, so each worker fills its molecules' rows.
 * Any other input is handed to aimx_csr_host_build. */
int aimx_collate_csr(aimx_collator* c, const int64_t* edges, int64_t E, const int64_t* batch, int64_t N, int64_t G,
                     int32_t hops, int32_t* fwd_rowptr, int32_t* fwd_col, int32_t* bwd_rowptr, int32_t* bwd_col,
                     int32_t* graph_rowptr, int32_t* graph_col);

#ifdef __cplusplus
}
#endif

#endif /* AIMX_HOST_H_ */
