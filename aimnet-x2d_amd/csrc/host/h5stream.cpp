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
// pickle_lite.h (data only; nothing executes) in parallel worker threads and packed into a
// store (aimx_store_create_hops) in one pass, with no Python objects per molecule.
#include <hdf5.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <exception>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/aimx_h5.h"
#include "../../../include/aimx_host.h"
#include "pickle_lite.h"

using aimx_pickle::Kind;
using aimx_pickle::Obj;

namespace {

const char* kFeatureKeys[4] = {"atom_type", "hydrogen_count", "degree", "hybridization"};

// One decoded molecule in flat form.
struct Mol {
  int32_t n_atoms = 0;
  std::vector<int32_t> feats;    // [n_atoms, 4]
  std::vector<int64_t> hop_len;  // [n_hops]
  std::vector<int32_t> pairs;    // (u, w) rows, hop-major
  std::vector<float> target;     // [n_tasks]
  float charge = 0.f;
};

// Reference _build_data_object (molecular.py:253-329): None or a record without 'precomputed' is
// skipped. Beyond that, a record this store cannot represent is reported invalid instead of
// raising later in collate: fewer than n_hops hop arrays, a hop array not [2, E], a target of
// the wrong length, atom indices out of range, a feature array of the wrong length.
bool decode_record(const uint8_t* p, size_t n, int32_t n_hops, int32_t n_tasks, Mol* m) {
  aimx_pickle::Decoder dec;
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
  m->n_atoms = (int32_t)na;
  m->feats.resize(size_t(na) * 4);
  for (int k = 0; k < 4; ++k) {
    if (col[k]->shape[0] != na) return false;
    int32_t* dst = m->feats.data() + k;
    if (!aimx_pickle::with_ints(*col[k], [&](auto get) {
          for (int64_t i = 0; i < na; ++i) dst[4 * i] = (int32_t)get(i);
        }))
      return false;
  }
  const Obj* mh = pre->get("multi_hop_edges");
  if (!mh || (mh->k != Kind::List && mh->k != Kind::Tuple) || (int64_t)mh->items.size() < n_hops) return false;
  m->hop_len.assign(n_hops, 0);
  int64_t tot = 0;
  for (int32_t h = 0; h < n_hops; ++h) {
    const Obj& e = *mh->items[h];
    if (e.k != Kind::Array || e.shape.size() != 2 || e.shape[0] != 2) return false;
    // a first-visit pair list holds at most na * (na - 1) pairs (features.py:97-150); the
    // decoder already checked the payload holds exactly 2 * E elements
    const int64_t E = e.shape[1];
    if (E < 0 || E > na * std::max<int64_t>(na - 1, 0)) return false;
    m->hop_len[h] = E;
    tot += E;
  }
  m->pairs.resize(size_t(2 * tot));
  int32_t* dst = m->pairs.data();
  for (int32_t h = 0; h < n_hops; ++h) {
    const Obj& e = *mh->items[h];
    const int64_t E = e.shape[1];
    bool in_range = true;
    // element (r, q) of a [2, E] array: C order r*E + q, Fortran order q*2 + r
    if (!aimx_pickle::with_ints(e, [&](auto get) {
          for (int64_t q = 0; q < E; ++q) {
            const int64_t u = get(e.fortran ? 2 * q : q), w = get(e.fortran ? 2 * q + 1 : E + q);
            in_range &= u >= 0 && u < na && w >= 0 && w < na;
            dst[2 * q] = (int32_t)u;
            dst[2 * q + 1] = (int32_t)w;
          }
        }) ||
        !in_range)
      return false;
    dst += 2 * E;
  }
  double tc = 0.0;
  if (!aimx_pickle::as_f64(pre->get("total_charge"), &tc)) return false;
  m->charge = (float)tc;
  const Obj* t = root->get("target");
  m->target.assign(n_tasks, 0.f);
  if (!t) return false;
  if (t->k == Kind::List || t->k == Kind::Tuple) {
    if ((int64_t)t->items.size() != n_tasks) return false;
    for (int32_t k = 0; k < n_tasks; ++k) {
      double v;
      if (!aimx_pickle::as_f64(t->items[k].get(), &v)) return false;
      m->target[k] = (float)v;
    }
  } else if (t->k == Kind::Array && t->numel() == n_tasks && n_tasks > 1) {
    for (int32_t k = 0; k < n_tasks; ++k) {
      double v;
      if (!aimx_pickle::elem_f64(*t, k, &v)) return false;
      m->target[k] = (float)v;
    }
  } else {
    double v;
    if (n_tasks != 1 || !aimx_pickle::as_f64(t, &v)) return false;
    m->target[0] = (float)v;
  }
  return true;
}

template <typename F>
void parallel_for(int64_t n, int threads, F&& f) {
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n));
  if (threads == 1) {
    f(0, n);
    return;
  }
  // an exception inside a worker (e.g. bad_alloc) must not reach std::terminate: the first one
  // is rethrown on the calling thread after every worker joined
  std::vector<std::thread> th;
  std::exception_ptr first;
  std::mutex mu;
  for (int t = 0; t < threads; ++t) {
    const int64_t lo = n * t / threads, hi = n * (t + 1) / threads;
    th.emplace_back([&f, &first, &mu, lo, hi] {
      try {
        f(lo, hi);
      } catch (...) {
        std::lock_guard<std::mutex> g(mu);
        if (!first) first = std::current_exception();
      }
    });
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

}  // namespace

struct aimx_h5_reader {
  hid_t file = -1, data = -1, space = -1, memtype = -1;
  int64_t n_records = 0;
  std::vector<int32_t> index_map;
  AimxH5Info info{};
  ~aimx_h5_reader() {
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
  std::vector<Mol> mols;
  std::vector<uint8_t> ok;
  try {
    mols.resize(size_t(n));
    ok.assign(size_t(n), 0);
    if (n > 0) {
      std::vector<hvl_t> raw(static_cast<size_t>(n));
      // records index_map[pos[k]] in request order: one hyperslab when contiguous, else a point list
      std::vector<hsize_t> coord(static_cast<size_t>(n));
      bool run = true;
      for (int64_t k = 0; k < n; ++k) {
        coord[k] = (hsize_t)r->index_map[pos[k]];
        if (k && coord[k] != coord[k - 1] + 1) run = false;
      }
      herr_t sel;
      if (run) {
        hsize_t start[1] = {coord[0]}, count[1] = {(hsize_t)n};
        sel = H5Sselect_hyperslab(r->space, H5S_SELECT_SET, start, nullptr, count, nullptr);
      } else {
        sel = H5Sselect_elements(r->space, H5S_SELECT_SET, (size_t)n, coord.data());
      }
      hsize_t md[1] = {(hsize_t)n};
      hid_t ms = H5Screate_simple(1, md, nullptr);
      if (sel < 0 || H5Dread(r->data, r->memtype, ms, r->space, H5P_DEFAULT, raw.data()) < 0) {
        H5Sclose(ms);
        return AIMX_H5_EIO;
      }
      parallel_for(n, n_threads, [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; ++k)
          ok[k] = decode_record((const uint8_t*)raw[k].p, raw[k].len, n_hops, n_tasks, &mols[k]);
      });
      H5Dvlen_reclaim(r->memtype, ms, H5P_DEFAULT, raw.data());
      H5Sclose(ms);
    }
    // pack the valid molecules (request order) into the store's flat arrays
    int64_t nv = 0, na = 0, np = 0;
    for (int64_t k = 0; k < n; ++k)
      if (ok[k]) {
        ++nv;
        na += mols[k].n_atoms;
        np += (int64_t)mols[k].pairs.size() / 2;
      }
    std::vector<int64_t> atom_ptr(size_t(nv) + 1, 0), hop_ptr(size_t(nv) * n_hops + 1, 0);
    std::vector<int32_t> feats(size_t(na) * 4), pairs(size_t(np) * 2);
    std::vector<float> targets(size_t(nv) * n_tasks), charge(static_cast<size_t>(nv));
    int64_t m = 0, ao = 0, po = 0;
    for (int64_t k = 0; k < n; ++k) {
      if (!ok[k]) continue;
      const Mol& x = mols[k];
      std::copy(x.feats.begin(), x.feats.end(), feats.begin() + ao * 4);
      ao += x.n_atoms;
      atom_ptr[m + 1] = ao;
      for (int32_t h = 0; h < n_hops; ++h) hop_ptr[m * n_hops + h + 1] = hop_ptr[m * n_hops + h] + x.hop_len[h];
      std::copy(x.pairs.begin(), x.pairs.end(), pairs.begin() + po * 2);
      po += (int64_t)x.pairs.size() / 2;
      std::copy(x.target.begin(), x.target.end(), targets.begin() + m * n_tasks);
      charge[m] = x.charge;
      if (valid_pos) valid_pos[m] = pos[k];
      ++m;
    }
    if (n_valid) *n_valid = nv;
    return aimx_store_create_hops(nv, atom_ptr.data(), feats.data(), 4, n_hops, hop_ptr.data(), pairs.data(),
                                  targets.data(), n_tasks, charge.data(), out);
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
  Mol m;
  try {
    if (!decode_record(bytes, size_t(n), n_hops, n_tasks, &m)) return 0;
  } catch (const std::bad_alloc&) {
    return AIMX_HOST_ENOMEM;
  }
  if (n_atoms) *n_atoms = m.n_atoms;
  if (n_pairs) *n_pairs = (int64_t)m.pairs.size() / 2;
  return 1;
}

}  // extern "C"
