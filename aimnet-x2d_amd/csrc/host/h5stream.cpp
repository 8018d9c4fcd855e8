// HDF5 molecule stream (host C++): the reference's on-disk dataset format, read and written
// natively, feeding the batch builder's molecule store.
//
// Format (reference writer src/datasets/features.py:381-431, 537-596; reader
// src/datasets/molecular.py:102-329, HDF5MolecularIterableDataset):
//   /data          1-D variable-length uint8 (vlen of H5T_STD_U8LE): one pickled dict per molecule,
//                  {'smiles': str, 'target': float | list, 'precomputed': compute_all's dict}
//                  (pickle.dumps(None) for an unparseable SMILES)
//   /index_map     1-D int32, record order (identity when written)
//   /metadata      group; attrs num_samples (int64), task_type (str), max_hops (int64),
//                  preprocessing_applied (bool), estimated_valid_pct (float64);
//                  subgroup sae (attrs applied (bool), note (str)); optional target_columns (str[])
// h5py is not part of this toolchain; the library is the HDF5 C library itself (1.10, as h5py
// links), so the files are the ones h5py reads and writes. Records are decoded by
// pickle_lite.h (data only; nothing executes) in parallel worker threads, in file order, and
// written into a new store (store.h) in request order, with no Python objects per molecule.
#include <fcntl.h>
#include <hdf5.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../../include/aimx_h5.h"
#include "../../../include/aimx_host.h"
#include "pickle_lite.h"
#include "store.h"

using aimx_pickle::Kind;
using aimx_pickle::Obj;

namespace {

const char* kFeatureKeys[4] = {"atom_type", "hydrogen_count", "degree", "hybridization"};

// Decoded molecules in flat form, appended record after record (one Part per worker, kept by the
// reader between reads: no allocation per molecule or per read once the buffers have grown).
struct Part {
  std::vector<int32_t> n_atoms;  // per molecule
  std::vector<int32_t> feats;    // [atoms, 4]
  std::vector<int64_t> hop_len;  // [molecules, n_hops]
  std::vector<uint16_t> pairs;   // (u, w) rows, hop-major per molecule (local indices < 65536)
  std::vector<float> target;     // [molecules, n_tasks]
  std::vector<float> charge;     // per molecule
  std::vector<int64_t> req;      // request index of each molecule
  void clear() {
    n_atoms.clear();
    feats.clear();
    hop_len.clear();
    pairs.clear();
    target.clear();
    charge.clear();
    req.clear();
  }
};

// Reference _build_data_object (molecular.py:253-329): None or a record without 'precomputed' is
// skipped. Beyond that, a record this store cannot represent is reported invalid instead of
// raising later in collate: fewer than n_hops hop arrays, a hop array not [2, E], a target of
// the wrong length, atom indices out of range, a feature array of the wrong length.
// Appends the molecule to `m` and returns true, or leaves `m` as it was and returns false.
bool decode_record(const uint8_t* p, size_t n, int32_t n_hops, int32_t n_tasks, Part* m) {
  thread_local aimx_pickle::Decoder dec;  // arena reused record after record
  std::string err;
  auto root = dec.decode(p, n, &err);
  if (!root || root->k != Kind::Dict) return false;
  const Obj* pre = root->get("precomputed");
  if (!pre || pre->k != Kind::Dict) return false;
  const Obj* af = pre->get("atom_features");
  if (!af || af->k != Kind::Dict) return false;
  const Obj* col[4];
  for (int k = 0; k < 4; ++k) {
    col[k] = af->get(kFeatureKeys[k]);
    if (!col[k] || col[k]->k != Kind::Array || col[k]->shape.size() != 1) return false;
  }
  const int64_t na = col[0]->shape[0];
  if (na < 0 || na > 65535) return false;
  const Obj* mh = pre->get("multi_hop_edges");
  if (!mh || (mh->k != Kind::List && mh->k != Kind::Tuple) || (int64_t)mh->items.size() < n_hops) return false;
  int64_t tot = 0;
  for (int32_t h = 0; h < n_hops; ++h) {
    const Obj& e = *mh->items[h];
    if (e.k != Kind::Array || e.shape.size() != 2 || e.shape[0] != 2) return false;
    // a first-visit pair list holds at most na * (na - 1) pairs (features.py:97-150); the
    // decoder already checked the payload holds exactly 2 * E elements
    const int64_t E = e.shape[1];
    if (E < 0 || E > na * std::max<int64_t>(na - 1, 0)) return false;
    tot += E;
  }
  double tc = 0.0;
  if (!aimx_pickle::as_f64(pre->get("total_charge"), &tc)) return false;
  float tv[64];
  std::vector<float> tbig;
  float* tg = n_tasks <= 64 ? tv : (tbig.resize(n_tasks), tbig.data());
  const Obj* t = root->get("target");
  if (!t) return false;
  if (t->k == Kind::List || t->k == Kind::Tuple) {
    if ((int64_t)t->items.size() != n_tasks) return false;
    for (int32_t k = 0; k < n_tasks; ++k) {
      double v;
      if (!aimx_pickle::as_f64(t->items[k], &v)) return false;
      tg[k] = (float)v;
    }
  } else if (t->k == Kind::Array && t->numel() == n_tasks && n_tasks > 1) {
    for (int32_t k = 0; k < n_tasks; ++k) {
      double v;
      if (!aimx_pickle::elem_f64(*t, k, &v)) return false;
      tg[k] = (float)v;
    }
  } else {
    double v;
    if (n_tasks != 1 || !aimx_pickle::as_f64(t, &v)) return false;
    tg[0] = (float)v;
  }
  // everything but the array contents checked: append, rolling back on a bad element
  const size_t f0 = m->feats.size(), p0 = m->pairs.size();
  m->feats.resize(f0 + size_t(na) * 4);
  bool good = true;
  for (int k = 0; k < 4 && good; ++k) {
    if (col[k]->shape[0] != na) {
      good = false;
      break;
    }
    int32_t* dst = m->feats.data() + f0 + k;
    good = aimx_pickle::with_ints(*col[k], [&](auto get) {
      for (int64_t i = 0; i < na; ++i) dst[4 * i] = (int32_t)get(i);
    });
  }
  if (good) m->pairs.resize(p0 + size_t(2 * tot));
  uint16_t* dst = m->pairs.data() + p0;
  for (int32_t h = 0; h < n_hops && good; ++h) {
    const Obj& e = *mh->items[h];
    const int64_t E = e.shape[1];
    bool in_range = true;
    // element (r, q) of a [2, E] array: C order r*E + q, Fortran order q*2 + r
    good = aimx_pickle::with_ints(e, [&](auto get) {
      for (int64_t q = 0; q < E; ++q) {
        const int64_t u = get(e.fortran ? 2 * q : q), w = get(e.fortran ? 2 * q + 1 : E + q);
        in_range &= u >= 0 && u < na && w >= 0 && w < na;
        dst[2 * q] = (uint16_t)u;
        dst[2 * q + 1] = (uint16_t)w;
      }
    }) && in_range;
    dst += 2 * E;
  }
  if (!good) {
    m->feats.resize(f0);
    m->pairs.resize(p0);
    return false;
  }
  m->n_atoms.push_back((int32_t)na);
  for (int32_t h = 0; h < n_hops; ++h) m->hop_len.push_back(mh->items[h]->shape[1]);
  m->target.insert(m->target.end(), tg, tg + n_tasks);
  m->charge.push_back((float)tc);
  return true;
}

// f(worker, lo, hi) on `threads` threads over contiguous ranges of [0, n), in worker order
template <typename F>
void parallel_for(int64_t n, int threads, F&& f) {
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n));
  if (threads == 1) {
    f(0, 0, n);
    return;
  }
  // an exception inside a worker (e.g. bad_alloc) must not reach std::terminate: the first one
  // is rethrown on the calling thread after every worker joined
  std::vector<std::thread> th;
  std::exception_ptr first;
  std::mutex mu;
  auto work = [&f, &first, &mu](int t, int64_t lo, int64_t hi) {
    try {
      f(t, lo, hi);
    } catch (...) {
      std::lock_guard<std::mutex> g(mu);
      if (!first) first = std::current_exception();
    }
  };
  for (int t = 0; t < threads; ++t) {
    const int64_t lo = n * t / threads, hi = n * (t + 1) / threads;
    bool spawned = false;
    try {
      th.emplace_back(work, t, lo, hi);
      spawned = true;
    } catch (const std::system_error&) {  // no more threads on this host: run the range here
    }
    if (!spawned) work(t, lo, hi);
  }
  for (auto& x : th) x.join();
  if (first) std::rethrow_exception(first);
}

// scalar attribute helpers (missing attribute: false)
bool attr_i64(hid_t obj, const char* name, int64_t* out) {
  if (H5Aexists(obj, name) <= 0) return false;
  hid_t a = H5Aopen(obj, name, H5P_DEFAULT);
  if (a < 0) return false;
  hid_t ft = H5Aget_type(a);
  bool ok = false;
  if (H5Tget_class(ft) == H5T_ENUM) {  // h5py bool: enum over int8 {FALSE, TRUE}
    hid_t nt = H5Tget_native_type(ft, H5T_DIR_ASCEND);
    unsigned char buf[8] = {0};
    const size_t sz = H5Tget_size(nt);
    if (sz <= 8 && H5Aread(a, nt, buf) >= 0) {
      int64_t v = 0;
      std::memcpy(&v, buf, sz);
      *out = v;
      ok = true;
    }
    H5Tclose(nt);
  } else if (H5Tget_class(ft) == H5T_INTEGER || H5Tget_class(ft) == H5T_FLOAT) {
    long long v = 0;
    ok = H5Aread(a, H5T_NATIVE_LLONG, &v) >= 0;
    *out = v;
  }
  H5Tclose(ft);
  H5Aclose(a);
  return ok;
}

bool attr_str(hid_t obj, const char* name, std::string* out) {
  if (H5Aexists(obj, name) <= 0) return false;
  hid_t a = H5Aopen(obj, name, H5P_DEFAULT);
  if (a < 0) return false;
  hid_t ft = H5Aget_type(a);
  bool ok = false;
  if (H5Tget_class(ft) == H5T_STRING) {
    if (H5Tis_variable_str(ft) > 0) {
      hid_t mt = H5Tcopy(H5T_C_S1);
      H5Tset_size(mt, H5T_VARIABLE);
      H5Tset_cset(mt, H5Tget_cset(ft));
      char* s = nullptr;
      if (H5Aread(a, mt, &s) >= 0 && s) {
        *out = s;
        ok = true;
        hid_t sp = H5Aget_space(a);
        H5Dvlen_reclaim(mt, sp, H5P_DEFAULT, &s);
        H5Sclose(sp);
      }
      H5Tclose(mt);
    } else {
      const size_t sz = H5Tget_size(ft);
      std::string buf(sz + 1, '\0');
      if (H5Aread(a, ft, &buf[0]) >= 0) {
        buf.resize(std::strlen(buf.c_str()));
        *out = buf;
        ok = true;
      }
    }
  }
  H5Tclose(ft);
  H5Aclose(a);
  return ok;
}

void set_attr_i64(hid_t obj, const char* name, int64_t v) {
  hid_t sp = H5Screate(H5S_SCALAR);
  hid_t a = H5Acreate2(obj, name, H5T_STD_I64LE, sp, H5P_DEFAULT, H5P_DEFAULT);
  long long x = v;
  H5Awrite(a, H5T_NATIVE_LLONG, &x);
  H5Aclose(a);
  H5Sclose(sp);
}

void set_attr_f64(hid_t obj, const char* name, double v) {
  hid_t sp = H5Screate(H5S_SCALAR);
  hid_t a = H5Acreate2(obj, name, H5T_IEEE_F64LE, sp, H5P_DEFAULT, H5P_DEFAULT);
  H5Awrite(a, H5T_NATIVE_DOUBLE, &v);
  H5Aclose(a);
  H5Sclose(sp);
}

hid_t bool_type() {  // h5py's numpy.bool_ mapping
  hid_t t = H5Tenum_create(H5T_NATIVE_INT8);
  signed char f = 0, tr = 1;
  H5Tenum_insert(t, "FALSE", &f);
  H5Tenum_insert(t, "TRUE", &tr);
  return t;
}

void set_attr_bool(hid_t obj, const char* name, bool v) {
  hid_t sp = H5Screate(H5S_SCALAR);
  hid_t t = bool_type();
  hid_t a = H5Acreate2(obj, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
  signed char x = v ? 1 : 0;
  H5Awrite(a, t, &x);
  H5Aclose(a);
  H5Tclose(t);
  H5Sclose(sp);
}

hid_t vlen_str_type() {  // h5py's str: variable-length UTF-8
  hid_t t = H5Tcopy(H5T_C_S1);
  H5Tset_size(t, H5T_VARIABLE);
  H5Tset_cset(t, H5T_CSET_UTF8);
  return t;
}

void set_attr_str(hid_t obj, const char* name, const char* v) {
  hid_t sp = H5Screate(H5S_SCALAR);
  hid_t t = vlen_str_type();
  hid_t a = H5Acreate2(obj, name, t, sp, H5P_DEFAULT, H5P_DEFAULT);
  H5Awrite(a, t, &v);
  H5Aclose(a);
  H5Tclose(t);
  H5Sclose(sp);
}


template <typename T>
T le(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

// Record bytes of /data element `coord` straight from the mapped file (HDF5 file format: a vlen
// element on disk is its length, the address of a global heap collection and the object's index in
// it; a collection is "GCOL", version 1, 3 reserved bytes, its size, then objects of
// {uint16 index, uint16 refcount, uint32 reserved, uint64 size, data padded to 8 bytes} up to a
// free-space object of index 0). 1: found; 0: an empty element; -1: structure out of bounds.
int direct_record(const uint8_t* map, size_t size, uint64_t desc, uint64_t base, int64_t coord, const uint8_t** p,
                  size_t* n) {
  const uint64_t d = desc + 16 * uint64_t(coord);
  if (d + 16 > size) return -1;
  const uint32_t len = le<uint32_t>(map + d);
  const uint64_t addr = le<uint64_t>(map + d + 4);
  const uint32_t idx = le<uint32_t>(map + d + 12);
  if (len == 0) return 0;
  const uint64_t c = addr + base;
  if (c > size || size - c < 16 || std::memcmp(map + c, "GCOL", 4) != 0 || map[c + 4] != 1) return -1;
  const uint64_t csize = le<uint64_t>(map + c + 8);
  if (csize < 16 || csize > size - c) return -1;
  uint64_t o = c + 16;
  const uint64_t end = c + csize;
  while (o + 16 <= end) {
    const uint16_t k = le<uint16_t>(map + o);
    const uint64_t sz = le<uint64_t>(map + o + 8);
    if (k == 0 || sz > end - o - 16) return -1;
    if (k == idx) {
      if (sz != len) return -1;
      *p = map + o + 16;
      *n = size_t(sz);
      return 1;
    }
    o += 16 + ((sz + 7) & ~uint64_t(7));
  }
  return -1;
}


}  // namespace

struct aimx_h5_reader {
  hid_t file = -1, data = -1, space = -1, memtype = -1;
  int64_t n_records = 0;
  std::vector<int32_t> index_map;
  AimxH5Info info{};
  // direct path: the file mapped read-only; /data's element k is the 16-byte vlen descriptor at
  // desc + 16 k (uint32 length, uint64 global-heap collection address, uint32 object index)
  const uint8_t* map = nullptr;
  size_t map_size = 0;
  uint64_t desc = 0, addr_base = 0;
  // the mapped file's identity at open (re-checked before every direct read: a file replaced,
  // truncated or rewritten since then is read through H5Dread instead of a stale or short mapping)
  int map_fd = -1;
  struct stat map_st {};
  std::vector<Part> parts;  // decode buffers, reused read after read (one read at a time per handle)
  ~aimx_h5_reader() {
    if (map) munmap(const_cast<uint8_t*>(map), map_size);
    if (map_fd >= 0) ::close(map_fd);
    if (memtype >= 0) H5Tclose(memtype);
    if (space >= 0) H5Sclose(space);
    if (data >= 0) H5Dclose(data);
    if (file >= 0) H5Fclose(file);
  }
};

struct aimx_h5_writer {
  hid_t file = -1, data = -1, space = -1, memtype = -1, meta = -1;
  int64_t n = 0;
  ~aimx_h5_writer() {
    if (memtype >= 0) H5Tclose(memtype);
    if (space >= 0) H5Sclose(space);
    if (data >= 0) H5Dclose(data);
    if (meta >= 0) H5Gclose(meta);
    if (file >= 0) H5Fclose(file);
  }
};

// Map the file for the direct path when /data is one contiguous run of 16-byte descriptors in an
// 8-byte-address file, and keep it only if the records it finds equal H5Dread's for a sample of
// elements (first, last and spread between). Any doubt leaves the H5Dread path in place.
static std::atomic<int> g_allow_direct{1};

extern "C" void aimx_h5_set_direct(int32_t allow) { g_allow_direct.store(allow ? 1 : 0); }

static void try_direct(aimx_h5_reader* r, const char* path) {
  if (!g_allow_direct.load()) return;
  if (r->n_records <= 0) return;
  hid_t fcpl = H5Fget_create_plist(r->file);
  size_t sa = 0, ss = 0;
  hsize_t ub = 0;
  const bool sizes = fcpl >= 0 && H5Pget_sizes(fcpl, &sa, &ss) >= 0 && H5Pget_userblock(fcpl, &ub) >= 0;
  if (fcpl >= 0) H5Pclose(fcpl);
  if (!sizes || sa != 8 || ss != 8) return;
  hid_t dcpl = H5Dget_create_plist(r->data);
  const bool contiguous = dcpl >= 0 && H5Pget_layout(dcpl) == H5D_CONTIGUOUS;
  if (dcpl >= 0) H5Pclose(dcpl);
  const haddr_t off = H5Dget_offset(r->data);
  if (!contiguous || off == HADDR_UNDEF) return;
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return;
  struct stat st;
  void* m = MAP_FAILED;
  if (fstat(fd, &st) == 0 && st.st_size > 0) m = mmap(nullptr, size_t(st.st_size), PROT_READ, MAP_PRIVATE, fd, 0);
  if (m == MAP_FAILED) {
    ::close(fd);
    return;
  }
  const uint8_t* map = static_cast<const uint8_t*>(m);
  const size_t size = size_t(st.st_size);
  std::vector<hsize_t> sample;
  const int64_t N = r->n_records;
  for (int64_t j = 0; j < 63 && j < N; ++j) sample.push_back(hsize_t(N <= 63 ? j : j * (N - 1) / 62));
  std::vector<hvl_t> raw(sample.size());
  bool ok = H5Sselect_elements(r->space, H5S_SELECT_SET, sample.size(), sample.data()) >= 0;
  hsize_t md[1] = {(hsize_t)sample.size()};
  hid_t ms = H5Screate_simple(1, md, nullptr);
  ok = ok && H5Dread(r->data, r->memtype, ms, r->space, H5P_DEFAULT, raw.data()) >= 0;
  uint64_t base_found = ~uint64_t(0);
  if (ok) {
    // HDF5 addresses are relative to the superblock (after any user block): try both readings
    for (uint64_t base : {uint64_t(0), uint64_t(ub)}) {
      bool all = true;
      for (size_t j = 0; j < sample.size() && all; ++j) {
        const uint8_t* p = nullptr;
        size_t n = 0;
        const int rc = direct_record(map, size, uint64_t(off) + base, base, int64_t(sample[j]), &p, &n);
        all = (rc == 1 && n == raw[j].len && std::memcmp(p, raw[j].p, n) == 0) || (rc == 0 && raw[j].len == 0);
      }
      if (all) {
        base_found = base;
        break;
      }
    }
    H5Dvlen_reclaim(r->memtype, ms, H5P_DEFAULT, raw.data());
  }
  H5Sclose(ms);
  if (base_found == ~uint64_t(0)) {
    munmap(m, size);
    ::close(fd);
    return;
  }
  r->map_fd = fd;
  r->map_st = st;
  r->map = map;
  r->map_size = size;
  r->desc = uint64_t(off) + base_found;
  r->addr_base = base_found;
  r->info.direct_read = 1;
}

extern "C" {

int aimx_h5_open(const char* path, aimx_h5_reader** out) {
  if (!path || !out) return AIMX_HOST_EARG;
  *out = nullptr;
  H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);  // errors are returned, not printed
  auto* r = new (std::nothrow) aimx_h5_reader();
  if (!r) return AIMX_HOST_ENOMEM;
  r->file = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
  if (r->file < 0) {
    delete r;
    return AIMX_H5_EIO;
  }
  r->data = H5Dopen2(r->file, "data", H5P_DEFAULT);
  if (r->data < 0) {
    delete r;
    return AIMX_H5_EFORMAT;
  }
  r->space = H5Dget_space(r->data);
  hsize_t dims[1] = {0};
  if (H5Sget_simple_extent_ndims(r->space) != 1 || H5Sget_simple_extent_dims(r->space, dims, nullptr) != 1) {
    delete r;
    return AIMX_H5_EFORMAT;
  }
  {
    hid_t ft = H5Dget_type(r->data);
    const bool vlen = H5Tget_class(ft) == H5T_VLEN;
    H5Tclose(ft);
    if (!vlen) {
      delete r;
      return AIMX_H5_EFORMAT;
    }
  }
  r->memtype = H5Tvlen_create(H5T_NATIVE_UINT8);
  r->n_records = (int64_t)dims[0];
  // index_map (molecular.py:138-142: identity when absent)
  r->index_map.resize(size_t(r->n_records));
  bool have_map = false;
  if (H5Lexists(r->file, "index_map", H5P_DEFAULT) > 0) {
    hid_t d = H5Dopen2(r->file, "index_map", H5P_DEFAULT);
    hid_t sp = H5Dget_space(d);
    hsize_t md[1] = {0};
    if (H5Sget_simple_extent_ndims(sp) == 1 && H5Sget_simple_extent_dims(sp, md, nullptr) == 1 &&
        (int64_t)md[0] == r->n_records)
      have_map = H5Dread(d, H5T_NATIVE_INT32, H5S_ALL, H5S_ALL, H5P_DEFAULT, r->index_map.data()) >= 0;
    H5Sclose(sp);
    H5Dclose(d);
  }
  if (!have_map)
    for (int64_t i = 0; i < r->n_records; ++i) r->index_map[i] = (int32_t)i;
  for (int64_t i = 0; i < r->n_records; ++i)
    if (r->index_map[i] < 0 || r->index_map[i] >= r->n_records) {
      delete r;
      return AIMX_H5_EFORMAT;
    }
  // metadata (molecular.py:159-174: preprocessing flag from the attrs, else from sae/applied)
  AimxH5Info& I = r->info;
  I.direct_read = 0;
  try_direct(r, path);
  I.n_records = r->n_records;
  I.num_samples = r->n_records;
  I.max_hops = -1;
  I.preprocessing_applied = 0;
  I.task_type[0] = '\0';
  if (H5Lexists(r->file, "metadata", H5P_DEFAULT) > 0) {
    hid_t g = H5Gopen2(r->file, "metadata", H5P_DEFAULT);
    int64_t v;
    if (attr_i64(g, "num_samples", &v)) I.num_samples = v;
    if (attr_i64(g, "max_hops", &v)) I.max_hops = v;
    std::string s;
    if (attr_str(g, "task_type", &s)) std::snprintf(I.task_type, sizeof(I.task_type), "%s", s.c_str());
    if (attr_i64(g, "preprocessing_applied", &v)) {
      I.preprocessing_applied = v != 0;
    } else if (H5Lexists(g, "sae", H5P_DEFAULT) > 0) {
      hid_t sg = H5Gopen2(g, "sae", H5P_DEFAULT);
      if (attr_i64(sg, "applied", &v)) I.preprocessing_applied = v != 0;
      H5Gclose(sg);
    }
    H5Gclose(g);
  }
  *out = r;
  return AIMX_HOST_OK;
}

void aimx_h5_close(aimx_h5_reader* r) { delete r; }

int aimx_h5_info(const aimx_h5_reader* r, AimxH5Info* out) {
  if (!r || !out) return AIMX_HOST_EARG;
  *out = r->info;
  return AIMX_HOST_OK;
}

int aimx_h5_read_store(aimx_h5_reader* r, const int64_t* pos, int64_t n, int32_t n_hops, int32_t n_tasks,
                       int32_t n_threads, aimx_mol_store** out, int64_t* n_valid, int64_t* valid_pos) {
  if (!r || !out || n < 0 || (n > 0 && !pos) || n_hops < 1 || n_tasks < 1) return AIMX_HOST_EARG;
  *out = nullptr;
  for (int64_t k = 0; k < n; ++k)
    if (pos[k] < 0 || pos[k] >= r->n_records) return AIMX_HOST_EARG;
  const int P = (int)std::max<int64_t>(1, std::min<int64_t>(std::max(n_threads, 1), n));
  try {
    if ((int)r->parts.size() < P) r->parts.resize(size_t(P));
    // visit records in file order (the request sorted by record index, stable): the mapped file
    // and HDF5's point reads are walked forward; the store is still written in request order
    std::vector<int64_t> vis(static_cast<size_t>(n));
    for (int64_t k = 0; k < n; ++k) vis[k] = k;
    std::stable_sort(vis.begin(), vis.end(),
                     [&](int64_t a, int64_t b) { return r->index_map[pos[a]] < r->index_map[pos[b]]; });
    // decode visits [lo, hi) into part t
    auto decode_range = [&](int t, int64_t lo, int64_t hi, auto&& bytes_of) {
      Part& m = r->parts[size_t(t)];
      m.clear();
      for (int64_t j = lo; j < hi; ++j) {
        const uint8_t* p = nullptr;
        size_t len = 0;
        if (bytes_of(j, &p, &len) && decode_record(p, len, n_hops, n_tasks, &m)) m.req.push_back(vis[j]);
      }
    };
    if (r->map) {  // the file must still be the one mapped at open (path, size, modification time)
      struct stat now;
      if (fstat(r->map_fd, &now) != 0 || now.st_size != r->map_st.st_size || now.st_nlink == 0 ||
          now.st_mtim.tv_sec != r->map_st.st_mtim.tv_sec || now.st_mtim.tv_nsec != r->map_st.st_mtim.tv_nsec) {
        munmap(const_cast<uint8_t*>(r->map), r->map_size);
        r->map = nullptr;
        r->info.direct_read = 0;
      }
    }
    if (n > 0 && r->map) {
      // direct path: every worker finds and decodes its records in the mapped file (the file must
      // stay unmodified while a read is in progress: a change between the check above and the read
      // is not caught)
      std::atomic<bool> corrupt{false};
      parallel_for(n, P, [&](int t, int64_t lo, int64_t hi) {
        decode_range(t, lo, hi, [&](int64_t j, const uint8_t** p, size_t* len) {
          const int rc = direct_record(r->map, r->map_size, r->desc, r->addr_base, r->index_map[pos[vis[j]]], p, len);
          if (rc < 0) corrupt = true;
          return rc == 1;
        });
      });
      if (corrupt) return AIMX_H5_EFORMAT;
    } else if (n > 0) {
      // one hyperslab when the visits are a contiguous run, else a point list (already in file
      // order: HDF5 reads a sorted point list several times faster); raw[j] is visit j's record
      std::vector<hsize_t> coord(static_cast<size_t>(n));
      bool run = true;
      for (int64_t j = 0; j < n; ++j) {
        coord[j] = (hsize_t)r->index_map[pos[vis[j]]];
        if (j && coord[j] != coord[j - 1] + 1) run = false;
      }
      herr_t sel;
      if (run) {
        hsize_t start[1] = {coord[0]}, count[1] = {(hsize_t)n};
        sel = H5Sselect_hyperslab(r->space, H5S_SELECT_SET, start, nullptr, count, nullptr);
      } else {
        sel = H5Sselect_elements(r->space, H5S_SELECT_SET, (size_t)n, coord.data());
      }
      std::vector<hvl_t> raw(static_cast<size_t>(n));
      hsize_t md[1] = {(hsize_t)n};
      hid_t ms = H5Screate_simple(1, md, nullptr);
      if (sel < 0 || H5Dread(r->data, r->memtype, ms, r->space, H5P_DEFAULT, raw.data()) < 0) {
        H5Sclose(ms);
        return AIMX_H5_EIO;
      }
      try {
        parallel_for(n, P, [&](int t, int64_t lo, int64_t hi) {
          decode_range(t, lo, hi, [&](int64_t j, const uint8_t** p, size_t* len) {
            const hvl_t& v = raw[size_t(j)];
            *p = (const uint8_t*)v.p;
            *len = v.len;
            return v.len > 0;
          });
        });
      } catch (...) {
        H5Dvlen_reclaim(r->memtype, ms, H5P_DEFAULT, raw.data());
        H5Sclose(ms);
        throw;
      }
      H5Dvlen_reclaim(r->memtype, ms, H5P_DEFAULT, raw.data());
      H5Sclose(ms);
    }
    // request-order placement: molecule, atom and pair offsets of every valid request
    std::vector<int32_t> na_k(static_cast<size_t>(n), -1);
    std::vector<int64_t> np_k(static_cast<size_t>(n), 0);
    parallel_for(P, P, [&](int, int64_t lo, int64_t hi) {
      for (int64_t t = lo; t < hi; ++t) {
        const Part& m = r->parts[size_t(t)];
        for (size_t i = 0; i < m.req.size(); ++i) {
          int64_t q = 0;
          for (int32_t h = 0; h < n_hops; ++h) q += m.hop_len[i * n_hops + h];
          na_k[m.req[i]] = m.n_atoms[i];
          np_k[m.req[i]] = q;
        }
      }
    });
    std::vector<int64_t> mol_k(static_cast<size_t>(n)), atom_k(static_cast<size_t>(n)), pair_k(static_cast<size_t>(n));
    int64_t nv = 0, NA = 0, NP = 0;
    for (int64_t k = 0; k < n; ++k) {
      mol_k[k] = nv;
      atom_k[k] = NA;
      pair_k[k] = NP;
      if (na_k[k] >= 0) {
        ++nv;
        NA += na_k[k];
        NP += np_k[k];
      }
    }
    // the store, filled in place by the workers, each copying its own part's molecules
    auto* s = new aimx_mol_store();
    std::unique_ptr<aimx_mol_store> own(s);
    s->n_mols = nv;
    s->n_feat = 4;
    s->n_tasks = n_tasks;
    s->cached_hops = n_hops;
    s->atom_ptr.resize(size_t(nv) + 1);
    s->bond_ptr.assign(size_t(nv) + 1, 0);
    s->feats.resize(size_t(NA) * 4);
    s->targets.resize(size_t(nv) * n_tasks);
    s->charge.resize(size_t(nv));
    s->hop_len.resize(size_t(nv) * n_hops);
    s->pair_ptr.resize(size_t(nv) + 1);
    s->pairs.resize(size_t(NP) * 2);
    s->atom_ptr[0] = 0;
    s->pair_ptr[0] = 0;
    parallel_for(P, P, [&](int, int64_t lo, int64_t hi) {
      for (int64_t t = lo; t < hi; ++t) {
        const Part& m = r->parts[size_t(t)];
        int64_t fa = 0, fq = 0;  // this molecule's atom / pair offset in the part
        for (size_t i = 0; i < m.req.size(); ++i) {
          const int64_t k = m.req[i], mol = mol_k[k], na = na_k[k], nq = np_k[k];
          std::memcpy(&s->feats[size_t(atom_k[k]) * 4], &m.feats[size_t(fa) * 4], sizeof(int32_t) * 4 * na);
          std::memcpy(&s->pairs[size_t(pair_k[k]) * 2], &m.pairs[size_t(fq) * 2], sizeof(uint16_t) * 2 * nq);
          for (int32_t h = 0; h < n_hops; ++h) s->hop_len[mol * n_hops + h] = int32_t(m.hop_len[i * n_hops + h]);
          std::memcpy(&s->targets[size_t(mol) * n_tasks], &m.target[i * n_tasks], sizeof(float) * n_tasks);
          s->charge[mol] = m.charge[i];
          s->atom_ptr[mol + 1] = atom_k[k] + na;
          s->pair_ptr[mol + 1] = pair_k[k] + nq;
          if (valid_pos) valid_pos[mol] = pos[k];
          fa += na;
          fq += nq;
        }
      }
    });
    if (n_valid) *n_valid = nv;
    *out = own.release();
    return AIMX_HOST_OK;
  } catch (const std::bad_alloc&) {
    return AIMX_HOST_ENOMEM;
  }
}

int aimx_h5_writer_create(const char* path, int64_t n_records, const AimxH5Info* meta, aimx_h5_writer** out) {
  if (!path || !out || !meta || n_records < 0) return AIMX_HOST_EARG;
  *out = nullptr;
  H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
  auto* w = new (std::nothrow) aimx_h5_writer();
  if (!w) return AIMX_HOST_ENOMEM;
  w->n = n_records;
  w->file = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
  if (w->file < 0) {
    delete w;
    return AIMX_H5_EIO;
  }
  hsize_t dims[1] = {(hsize_t)n_records};
  w->space = H5Screate_simple(1, dims, nullptr);
  hid_t ft = H5Tvlen_create(H5T_STD_U8LE);
  w->data = H5Dcreate2(w->file, "data", ft, w->space, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
  H5Tclose(ft);
  w->memtype = H5Tvlen_create(H5T_NATIVE_UINT8);
  // index_map: identity (features.py:420-421)
  hid_t im = H5Dcreate2(w->file, "index_map", H5T_STD_I32LE, w->space, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
  herr_t st = -1;
  try {
    std::vector<int32_t> ident(static_cast<size_t>(n_records));
    for (int64_t i = 0; i < n_records; ++i) ident[i] = (int32_t)i;
    st = H5Dwrite(im, H5T_NATIVE_INT32, H5S_ALL, H5S_ALL, H5P_DEFAULT, ident.data());
  } catch (const std::bad_alloc&) {
  }
  H5Dclose(im);
  // metadata group and its attributes (features.py:423-435, 521-530)
  w->meta = H5Gcreate2(w->file, "metadata", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
  if (w->data < 0 || w->meta < 0 || st < 0) {
    delete w;
    return AIMX_H5_EIO;
  }
  set_attr_i64(w->meta, "num_samples", n_records);
  set_attr_str(w->meta, "task_type", meta->task_type);
  set_attr_i64(w->meta, "max_hops", meta->max_hops);
  set_attr_bool(w->meta, "preprocessing_applied", meta->preprocessing_applied != 0);
  hid_t sae = H5Gcreate2(w->meta, "sae", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
  set_attr_bool(sae, "applied", meta->preprocessing_applied != 0);
  if (meta->preprocessing_applied) set_attr_str(sae, "note", "Applied during preprocessing before HDF5 creation");
  H5Gclose(sae);
  *out = w;
  return AIMX_HOST_OK;
}

int aimx_h5_writer_put(aimx_h5_writer* w, int64_t start, int64_t count, const uint8_t* bytes,
                       const int64_t* offsets) {
  if (!w || start < 0 || count < 0 || start + count > w->n || (count > 0 && (!bytes || !offsets)))
    return AIMX_HOST_EARG;
  if (count == 0) return AIMX_HOST_OK;
  std::vector<hvl_t> v(static_cast<size_t>(count));
  for (int64_t k = 0; k < count; ++k) {
    if (offsets[k + 1] < offsets[k]) return AIMX_HOST_EARG;
    v[k].len = size_t(offsets[k + 1] - offsets[k]);
    v[k].p = (void*)(bytes + offsets[k]);
  }
  hsize_t s0[1] = {(hsize_t)start}, c0[1] = {(hsize_t)count};
  hid_t ms = H5Screate_simple(1, c0, nullptr);
  const bool ok = H5Sselect_hyperslab(w->space, H5S_SELECT_SET, s0, nullptr, c0, nullptr) >= 0 &&
                  H5Dwrite(w->data, w->memtype, ms, w->space, H5P_DEFAULT, v.data()) >= 0;
  H5Sclose(ms);
  return ok ? AIMX_HOST_OK : AIMX_H5_EIO;
}

int aimx_h5_writer_close(aimx_h5_writer* w, double estimated_valid_pct) {
  if (!w) return AIMX_HOST_EARG;
  set_attr_f64(w->meta, "estimated_valid_pct", estimated_valid_pct);
  const bool ok = H5Fflush(w->file, H5F_SCOPE_GLOBAL) >= 0;
  delete w;
  return ok ? AIMX_HOST_OK : AIMX_H5_EIO;
}

int32_t aimx_h5_decode_record(const uint8_t* bytes, int64_t n, int32_t n_hops, int32_t n_tasks, int32_t* n_atoms,
                              int64_t* n_pairs) {
  if (!bytes || n < 0 || n_hops < 1 || n_tasks < 1) return AIMX_HOST_EARG;
  Part m;
  try {
    if (!decode_record(bytes, size_t(n), n_hops, n_tasks, &m)) return 0;
  } catch (const std::bad_alloc&) {
    return AIMX_HOST_ENOMEM;
  }
  if (n_atoms) *n_atoms = m.n_atoms[0];
  if (n_pairs) *n_pairs = (int64_t)m.pairs.size() / 2;
  return 1;
}

}  // extern "C"
