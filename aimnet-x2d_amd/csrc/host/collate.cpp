// Native batch builder (host C++): multi-hop BFS pair lists + collate into caller buffers.
//
// Reference stages replaced:
//   src/datasets/features.py:82-95   build_numba_adjacency_list   (neighbours = nonzero columns of
//                                    the adjacency row, ascending, self-loops skipped)
//   src/datasets/features.py:97-150  compute_multi_hop_edges_bfs_numba (edge-space BFS: hop 1 in
//                                    (v, w) order; hop k expands the previous hop's pairs in order,
//                                    keeps first-visit (u, w) with w != u; stops at an empty hop)
//   src/datasets/molecular.py:339-458 MyBatch.from_data_list (hop arrays + atom offset, concat
//                                    molecule-major / hop-major, .t() -> [E, 2]; batch ids)
// Design: molecules are independent, so a batch is planned (per-molecule pair lists and prefix
// offsets) by a persistent worker pool over contiguous molecule ranges, then written straight into
// the caller's (pinned) buffers by the same workers — no intermediate Python objects and one
// contiguous write stream per worker.
#include "../../../include/aimx_host.h"
#include "store.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------------
// Worker pool: run(f) calls f(worker_id) on every worker (the caller is worker 0) and returns when
// all have finished. One job at a time (callers serialise per collator).
// ---------------------------------------------------------------------------------------------
class Pool {
 public:
  // A host that refuses more threads (EAGAIN under a pid / task limit) gets a smaller pool, not
  // std::terminate from a half-built thread vector.
  explicit Pool(int n) : n_(std::max(1, n)) {
    for (int i = 1; i < n_; ++i) {
      try {
        th_.emplace_back([this, i] { loop(i); });
      } catch (const std::system_error&) {
        n_ = i;
        break;
      }
    }
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  void run(const std::function<void(int)>& f) {
    if (n_ == 1) {
      f(0);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &f;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        f = job_;
      }
      (*f)(id);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

inline void split_range(int64_t n, int parts, int part, int64_t* lo, int64_t* hi) {
  int64_t q = n / parts, r = n % parts;
  *lo = part * q + std::min<int64_t>(part, r);
  *hi = *lo + q + (part < r ? 1 : 0);
}

// ---------------------------------------------------------------------------------------------
// BFS of one molecule. Scratch is reused across molecules by one worker.
// ---------------------------------------------------------------------------------------------
struct BfsScratch {
  std::vector<int32_t> deg, nptr, nbr;
  std::vector<uint8_t> visited;  // n x n (the reference's visited matrix)
  std::vector<int32_t> pairs;    // (u, w) interleaved, hop-major
  std::vector<int64_t> hop_count;
};

// Returns false on invalid bonds (index outside [0, n)).
bool bfs_molecule(int32_t n, const int32_t* bonds, int64_t nb, int32_t max_hops, BfsScratch& s) {
  s.pairs.clear();
  s.hop_count.assign(std::max(max_hops, 0), 0);
  if (n <= 0 || max_hops <= 0) return n >= 0;
  // adjacency lists = sorted unique nonzero columns of the symmetric adjacency, minus self
  s.deg.assign(n + 1, 0);
  for (int64_t b = 0; b < nb; ++b) {
    int32_t i = bonds[2 * b], j = bonds[2 * b + 1];
    if (i < 0 || j < 0 || i >= n || j >= n) return false;
    if (i == j) continue;
    s.deg[i]++;
    s.deg[j]++;
  }
  s.nptr.assign(n + 1, 0);
  for (int32_t v = 0; v < n; ++v) s.nptr[v + 1] = s.nptr[v] + s.deg[v];
  s.nbr.resize(s.nptr[n]);
  std::fill(s.deg.begin(), s.deg.end(), 0);
  for (int64_t b = 0; b < nb; ++b) {
    int32_t i = bonds[2 * b], j = bonds[2 * b + 1];
    if (i == j) continue;
    s.nbr[s.nptr[i] + s.deg[i]++] = j;
    s.nbr[s.nptr[j] + s.deg[j]++] = i;
  }
  // sort + unique each row in place, keep the new end in deg[]
  for (int32_t v = 0; v < n; ++v) {
    int32_t* a = s.nbr.data() + s.nptr[v];
    int32_t* e = a + s.deg[v];
    std::sort(a, e);
    s.deg[v] = int32_t(std::unique(a, e) - a);
  }
  s.visited.assign(size_t(n) * size_t(n), 0);
  uint8_t* vis = s.visited.data();
  // hop 1 (features.py:107-112)
  for (int32_t v = 0; v < n; ++v) {
    const int32_t* a = s.nbr.data() + s.nptr[v];
    for (int32_t k = 0; k < s.deg[v]; ++k) {
      int32_t w = a[k];
      uint8_t& f = vis[size_t(v) * n + w];
      if (!f) {
        f = 1;
        s.pairs.push_back(v);
        s.pairs.push_back(w);
      }
    }
  }
  s.hop_count[0] = int64_t(s.pairs.size() / 2);
  size_t f0 = 0, f1 = s.pairs.size();  // frontier = pairs[f0, f1)
  // hops 2..max_hops (features.py:122-145); an empty hop ends the BFS, later hops stay empty
  for (int32_t h = 1; h < max_hops; ++h) {
    for (size_t p = f0; p < f1; p += 2) {
      int32_t u = s.pairs[p], v = s.pairs[p + 1];
      const int32_t* a = s.nbr.data() + s.nptr[v];
      for (int32_t k = 0; k < s.deg[v]; ++k) {
        int32_t w = a[k];
        if (w == u) continue;
        uint8_t& f = vis[size_t(u) * n + w];
        if (!f) {
          f = 1;
          s.pairs.push_back(u);
          s.pairs.push_back(w);
        }
      }
    }
    size_t added = s.pairs.size() - f1;
    s.hop_count[h] = int64_t(added / 2);
    if (!added) break;
    f0 = f1;
    f1 = s.pairs.size();
  }
  return true;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Store
// ---------------------------------------------------------------------------------------------
struct aimx_collator {
  int32_t max_hops;
  Pool pool;
  std::vector<BfsScratch> scratch;  // per worker
  // plan
  const aimx_mol_store* store = nullptr;
  std::vector<int64_t> idx, atom_off, edge_off;  // [G+1] prefix offsets
  std::vector<int64_t> mol_pair_base;             // per molecule: offset into wpairs[worker]
  std::vector<std::vector<int32_t>> wpairs;        // per worker planned pairs (uncached store)
  std::vector<int32_t> mol_worker;
  int64_t G = 0, N = 0, E = 0;
  bool planned = false;
  std::vector<int32_t> csr_next_f, csr_next_b;  // aimx_collate_csr row cursors
  aimx_collator(int32_t h, int32_t t) : max_hops(h), pool(t), scratch(pool.size()), wpairs(pool.size()) {}
};

extern "C" {

const char* aimx_host_version(void) { return "aimx_host/0.1"; }

int64_t aimx_bfs_multi_hop(int32_t n_atoms, const int32_t* bonds, int64_t n_bonds, int32_t max_hops,
                           int32_t* pairs, int64_t cap, int64_t* hop_counts) {
  if (n_atoms < 0 || n_bonds < 0 || max_hops < 0 || cap < 0 || (n_bonds > 0 && !bonds)) return AIMX_HOST_EARG;
  BfsScratch s;
  try {
    if (!bfs_molecule(n_atoms, bonds, n_bonds, max_hops, s)) return AIMX_HOST_EARG;
  } catch (const std::bad_alloc&) {
    return AIMX_HOST_ENOMEM;
  }
  int64_t total = int64_t(s.pairs.size() / 2);
  if (hop_counts)
    for (int32_t h = 0; h < max_hops; ++h) hop_counts[h] = s.hop_count[h];
  if (pairs) std::memcpy(pairs, s.pairs.data(), sizeof(int32_t) * 2 * size_t(std::min(total, cap)));
  return total;
}

int aimx_store_create(int64_t n_mols, const int64_t* atom_ptr, const int64_t* bond_ptr, const int32_t* bonds,
                      const int32_t* feats, int32_t n_feat, const float* targets, int32_t n_tasks,
                      const float* total_charge, int32_t precompute_hops, int32_t n_threads,
                      aimx_mol_store** out) {
  if (!out || n_mols < 0 || !atom_ptr || !bond_ptr || n_feat < 0 || n_feat > 8 || n_tasks < 0 ||
      precompute_hops < 0)
    return AIMX_HOST_EARG;
  *out = nullptr;
  if (atom_ptr[0] != 0 || bond_ptr[0] != 0) return AIMX_HOST_EARG;
  for (int64_t m = 0; m < n_mols; ++m) {
    int64_t na = atom_ptr[m + 1] - atom_ptr[m];
    if (na < 0 || na > 65535 || bond_ptr[m + 1] < bond_ptr[m]) return AIMX_HOST_EARG;
  }
  int64_t NA = atom_ptr[n_mols], NB = bond_ptr[n_mols];
  if ((NB > 0 && !bonds) || (NA > 0 && n_feat > 0 && !feats)) return AIMX_HOST_EARG;
  aimx_mol_store* s = nullptr;
  try {
    s = new aimx_mol_store();
    s->n_mols = n_mols;
    s->n_feat = n_feat;
    s->n_tasks = n_tasks;
    s->atom_ptr.assign(atom_ptr, atom_ptr + n_mols + 1);
    s->bond_ptr.assign(bond_ptr, bond_ptr + n_mols + 1);
    if (NB) s->bonds.assign(bonds, bonds + 2 * NB);
    if (NA && n_feat) s->feats.assign(feats, feats + NA * n_feat);
    s->targets.assign(size_t(n_mols) * n_tasks, 0.f);
    if (targets && n_tasks) std::memcpy(s->targets.data(), targets, sizeof(float) * s->targets.size());
    s->charge.assign(n_mols, 0.f);
    if (total_charge) std::memcpy(s->charge.data(), total_charge, sizeof(float) * n_mols);
    for (int64_t m = 0; m < n_mols; ++m) {  // validate bonds once, here
      int64_t na = atom_ptr[m + 1] - atom_ptr[m];
      for (int64_t b = bond_ptr[m]; b < bond_ptr[m + 1]; ++b)
        if (bonds[2 * b] < 0 || bonds[2 * b] >= na || bonds[2 * b + 1] < 0 || bonds[2 * b + 1] >= na) {
          delete s;
          return AIMX_HOST_EARG;
        }
    }
    if (precompute_hops > 0) {
      const int32_t H = precompute_hops;
      s->cached_hops = H;
      s->hop_len.assign(size_t(n_mols) * H, 0);
      Pool pool(std::max(1, n_threads));
      const int P = pool.size();
      std::vector<std::vector<uint16_t>> part(P);
      std::vector<int64_t> lo(P), hi(P);
      pool.run([&](int w) {
        BfsScratch sc;
        split_range(n_mols, P, w, &lo[w], &hi[w]);
        for (int64_t m = lo[w]; m < hi[w]; ++m) {
          int32_t na = int32_t(atom_ptr[m + 1] - atom_ptr[m]);
          bfs_molecule(na, bonds + 2 * bond_ptr[m], bond_ptr[m + 1] - bond_ptr[m], H, sc);
          for (int32_t h = 0; h < H; ++h) s->hop_len[size_t(m) * H + h] = int32_t(sc.hop_count[h]);
          part[w].insert(part[w].end(), sc.pairs.begin(), sc.pairs.end());
        }
      });
      s->pair_ptr.assign(n_mols + 1, 0);
      for (int64_t m = 0; m < n_mols; ++m) {
        int64_t t = 0;
        for (int32_t h = 0; h < H; ++h) t += s->hop_len[size_t(m) * H + h];
        s->pair_ptr[m + 1] = s->pair_ptr[m] + t;
      }
      s->pairs.reserve(size_t(2 * s->pair_ptr[n_mols]));
      for (int w = 0; w < P; ++w) s->pairs.insert(s->pairs.end(), part[w].begin(), part[w].end());
    }
  } catch (const std::bad_alloc&) {
    delete s;
    return AIMX_HOST_ENOMEM;
  }
  *out = s;
  return AIMX_HOST_OK;
}

int aimx_store_create_hops(int64_t n_mols, const int64_t* atom_ptr, const int32_t* feats, int32_t n_feat,
                           int32_t n_hops, const int64_t* hop_ptr, const int32_t* pairs, const float* targets,
                           int32_t n_tasks, const float* total_charge, aimx_mol_store** out) {
  if (!out || n_mols < 0 || !atom_ptr || n_feat < 0 || n_feat > 8 || n_tasks < 0 || n_hops < 1 || !hop_ptr)
    return AIMX_HOST_EARG;
  *out = nullptr;
  if (atom_ptr[0] != 0 || hop_ptr[0] != 0) return AIMX_HOST_EARG;
  const int64_t NH = n_mols * n_hops;
  for (int64_t m = 0; m < n_mols; ++m) {
    const int64_t na = atom_ptr[m + 1] - atom_ptr[m];
    if (na < 0 || na > 65535) return AIMX_HOST_EARG;
  }
  for (int64_t k = 0; k < NH; ++k)
    if (hop_ptr[k + 1] < hop_ptr[k]) return AIMX_HOST_EARG;
  const int64_t NA = atom_ptr[n_mols], NP = hop_ptr[NH];
  if ((NP > 0 && !pairs) || (NA > 0 && n_feat > 0 && !feats)) return AIMX_HOST_EARG;
  for (int64_t m = 0; m < n_mols; ++m) {  // local indices in range (the stored form is uint16)
    const int64_t na = atom_ptr[m + 1] - atom_ptr[m];
    for (int64_t q = hop_ptr[m * n_hops]; q < hop_ptr[(m + 1) * n_hops]; ++q)
      if (pairs[2 * q] < 0 || pairs[2 * q] >= na || pairs[2 * q + 1] < 0 || pairs[2 * q + 1] >= na)
        return AIMX_HOST_EARG;
  }
  aimx_mol_store* s = nullptr;
  try {
    s = new aimx_mol_store();
    s->n_mols = n_mols;
    s->n_feat = n_feat;
    s->n_tasks = n_tasks;
    s->atom_ptr.assign(atom_ptr, atom_ptr + n_mols + 1);
    s->bond_ptr.assign(n_mols + 1, 0);
    if (NA && n_feat) s->feats.assign(feats, feats + NA * n_feat);
    s->targets.assign(size_t(n_mols) * n_tasks, 0.f);
    if (targets && n_tasks) std::memcpy(s->targets.data(), targets, sizeof(float) * s->targets.size());
    s->charge.assign(n_mols, 0.f);
    if (total_charge) std::memcpy(s->charge.data(), total_charge, sizeof(float) * n_mols);
    s->cached_hops = n_hops;
    s->hop_len.resize(size_t(NH));
    for (int64_t k = 0; k < NH; ++k) s->hop_len[k] = int32_t(hop_ptr[k + 1] - hop_ptr[k]);
    s->pair_ptr.assign(n_mols + 1, 0);
    for (int64_t m = 0; m < n_mols; ++m) s->pair_ptr[m + 1] = hop_ptr[(m + 1) * n_hops];
    s->pairs.resize(size_t(2 * NP));
    for (int64_t q = 0; q < 2 * NP; ++q) s->pairs[q] = uint16_t(pairs[q]);
  } catch (const std::bad_alloc&) {
    delete s;
    return AIMX_HOST_ENOMEM;
  }
  *out = s;
  return AIMX_HOST_OK;
}

void aimx_store_destroy(aimx_mol_store* store) { delete store; }

int64_t aimx_store_num_molecules(const aimx_mol_store* s) { return s ? s->n_mols : AIMX_HOST_EARG; }

int64_t aimx_store_num_atoms(const aimx_mol_store* s, int64_t m) {
  if (!s || m < 0 || m >= s->n_mols) return AIMX_HOST_EARG;
  return s->atom_ptr[m + 1] - s->atom_ptr[m];
}

int aimx_store_atom_counts(const aimx_mol_store* s, int64_t* out) {
  if (!s || (s->n_mols > 0 && !out)) return AIMX_HOST_EARG;
  for (int64_t m = 0; m < s->n_mols; ++m) out[m] = s->atom_ptr[m + 1] - s->atom_ptr[m];
  return AIMX_HOST_OK;
}

int aimx_collator_create(int32_t max_hops, int32_t n_threads, aimx_collator** out) {
  if (!out || max_hops < 0) return AIMX_HOST_EARG;
  try {
    *out = new aimx_collator(max_hops, std::max(1, n_threads));
  } catch (const std::bad_alloc&) {
    *out = nullptr;
    return AIMX_HOST_ENOMEM;
  } catch (const std::system_error&) {
    *out = nullptr;
    return AIMX_HOST_ENOMEM;
  }
  return AIMX_HOST_OK;
}

void aimx_collator_destroy(aimx_collator* c) { delete c; }

int aimx_collate_plan(aimx_collator* c, const aimx_mol_store* s, const int64_t* idx, int64_t G, int64_t* n_atoms,
                      int64_t* n_edges) {
  if (!c || !s || G < 0 || (G > 0 && !idx)) return AIMX_HOST_EARG;
  c->planned = false;
  const bool cached = s->cached_hops > 0;
  if (cached && s->cached_hops < c->max_hops) return AIMX_HOST_EARG;
  for (int64_t g = 0; g < G; ++g)
    if (idx[g] < 0 || idx[g] >= s->n_mols) return AIMX_HOST_EARG;
  try {
    c->store = s;
    c->G = G;
    c->idx.assign(idx, idx + G);
    c->atom_off.assign(G + 1, 0);
    c->edge_off.assign(G + 1, 0);
    c->mol_pair_base.assign(G, 0);
    c->mol_worker.assign(G, 0);
    const int P = c->pool.size();
    const int32_t H = c->max_hops;
    std::vector<int64_t> cnt(G, 0);
    bool ok = true;
    if (cached) {
      const int32_t SH = s->cached_hops;
      for (int64_t g = 0; g < G; ++g) {
        const int32_t* hl = s->hop_len.data() + size_t(idx[g]) * SH;
        int64_t t = 0;
        for (int32_t h = 0; h < H; ++h) t += hl[h];
        cnt[g] = t;
      }
    } else {
      std::atomic<bool> good{true};
      c->pool.run([&](int w) {
        int64_t lo, hi;
        split_range(G, P, w, &lo, &hi);
        auto& dst = c->wpairs[w];
        dst.clear();
        BfsScratch& sc = c->scratch[w];
        for (int64_t g = lo; g < hi; ++g) {
          int64_t m = idx[g];
          int32_t na = int32_t(s->atom_ptr[m + 1] - s->atom_ptr[m]);
          if (!bfs_molecule(na, s->bonds.data() + 2 * s->bond_ptr[m], s->bond_ptr[m + 1] - s->bond_ptr[m], H, sc)) {
            good = false;
            return;
          }
          c->mol_pair_base[g] = int64_t(dst.size());
          c->mol_worker[g] = w;
          cnt[g] = int64_t(sc.pairs.size() / 2);
          dst.insert(dst.end(), sc.pairs.begin(), sc.pairs.end());
        }
      });
      ok = good;
    }
    if (!ok) return AIMX_HOST_EARG;
    for (int64_t g = 0; g < G; ++g) {
      c->atom_off[g + 1] = c->atom_off[g] + (s->atom_ptr[idx[g] + 1] - s->atom_ptr[idx[g]]);
      c->edge_off[g + 1] = c->edge_off[g] + cnt[g];
    }
    c->N = c->atom_off[G];
    c->E = c->edge_off[G];
  } catch (const std::bad_alloc&) {
    return AIMX_HOST_ENOMEM;
  }
  if (n_atoms) *n_atoms = c->N;
  if (n_edges) *n_edges = c->E;
  c->planned = true;
  return AIMX_HOST_OK;
}

int aimx_collate_write(aimx_collator* c, const AimxCollateOut* o) {
  if (!c || !o) return AIMX_HOST_EARG;
  if (!c->planned) return AIMX_HOST_ESTATE;
  const aimx_mol_store* s = c->store;
  const int64_t G = c->G, N = c->N, E = c->E;
  const bool pad = o->n_max > 0;
  if (pad && (o->n_max <= N || o->e_max < E || o->pad_mols < 1)) return AIMX_HOST_ESPACE;
  if (!o->edges || !o->batch) return AIMX_HOST_EARG;
  for (int32_t k = 0; k < s->n_feat; ++k)
    if (!o->feat[k]) return AIMX_HOST_EARG;
  const int P = c->pool.size();
  const int32_t SH = s->cached_hops, F = s->n_feat, T = s->n_tasks;
  const bool cached = SH > 0;
  c->pool.run([&](int w) {
    int64_t lo, hi;
    split_range(G, P, w, &lo, &hi);
    for (int64_t g = lo; g < hi; ++g) {
      const int64_t m = c->idx[g], a0 = c->atom_off[g], na = c->atom_off[g + 1] - a0;
      const int64_t src_a = s->atom_ptr[m];
      for (int64_t i = 0; i < na; ++i) o->batch[a0 + i] = g;
      for (int32_t k = 0; k < F; ++k) {
        int64_t* dst = o->feat[k] + a0;
        const int32_t* src = s->feats.data() + src_a * F + k;
        for (int64_t i = 0; i < na; ++i) dst[i] = src[i * F];
      }
      int64_t* e = o->edges + 2 * c->edge_off[g];
      const int64_t ne = c->edge_off[g + 1] - c->edge_off[g];
      if (cached) {
        // cached pairs are hop-major over SH hops; the first H hops are a prefix
        const uint16_t* p = s->pairs.data() + 2 * s->pair_ptr[m];
        for (int64_t q = 0; q < ne; ++q) {
          e[2 * q] = a0 + p[2 * q];
          e[2 * q + 1] = a0 + p[2 * q + 1];
        }
      } else {
        const int32_t* p = c->wpairs[c->mol_worker[g]].data() + c->mol_pair_base[g];
        for (int64_t q = 0; q < ne; ++q) {
          e[2 * q] = a0 + p[2 * q];
          e[2 * q + 1] = a0 + p[2 * q + 1];
        }
      }
      if (o->total_charges) o->total_charges[g] = s->charge[m];
      if (o->targets && T) std::memcpy(o->targets + g * T, s->targets.data() + m * T, sizeof(float) * T);
      if (o->n_atoms) o->n_atoms[g] = na;
    }
    if (!pad) return;
    // padding: worker w fills its share of slack atoms and slack edges
    const int64_t n_pad = o->n_max - N, q = n_pad / o->pad_mols, r = n_pad % o->pad_mols;
    int64_t plo, phi;
    split_range(n_pad, P, w, &plo, &phi);
    for (int64_t i = plo; i < phi; ++i) {
      // molecule of padding atom i: first r molecules have q+1 atoms, the rest q
      int64_t j = (i < r * (q + 1)) ? i / (q + 1) : r + (q ? (i - r * (q + 1)) / q : 0);
      o->batch[N + i] = G + j;
      for (int32_t k = 0; k < F; ++k) o->feat[k][N + i] = 0;
    }
    int64_t elo, ehi;
    split_range(o->e_max - E, P, w, &elo, &ehi);
    for (int64_t k = elo; k < ehi; ++k) {
      int64_t a = N + k % n_pad;
      o->edges[2 * (E + k)] = a;
      o->edges[2 * (E + k) + 1] = a;
    }
    if (w == 0) {
      for (int32_t j = 0; j < o->pad_mols; ++j) {
        if (o->total_charges) o->total_charges[G + j] = 0.f;
        if (o->targets && T) std::memset(o->targets + (G + j) * T, 0, sizeof(float) * T);
        if (o->n_atoms) o->n_atoms[G + j] = q + (j < r ? 1 : 0);
      }
    }
  });
  return AIMX_HOST_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Host CSR views (include/aimx_host.h): stable counting sorts, the host twin of csr.hip.
// ---------------------------------------------------------------------------------------------
namespace {

// rowptr[rows+1] and col[n] of the stable sort of items 0..n-1 by key(i) in [0, rows)
template <class Key, class Val>
void counting_csr(int64_t n, int64_t rows, Key key, Val val, int32_t* rowptr, int32_t* col) {
  std::fill(rowptr, rowptr + rows + 1, 0);
  for (int64_t i = 0; i < n; ++i) ++rowptr[key(i) + 1];
  for (int64_t r = 0; r < rows; ++r) rowptr[r + 1] += rowptr[r];
  std::vector<int32_t> next(rowptr, rowptr + rows);
  for (int64_t i = 0; i < n; ++i) col[next[key(i)]++] = val(i);
}

}  // namespace

extern "C" int aimx_csr_host_build(const int64_t* edges, int64_t E, const int64_t* batch, int64_t N, int64_t G,
                                   int32_t hops, int32_t* fwd_rowptr, int32_t* fwd_col, int32_t* bwd_rowptr,
                                   int32_t* bwd_col, int32_t* graph_rowptr, int32_t* graph_col) {
  const int64_t lim = int64_t(1) << 31;
  if (E < 0 || N < 0 || G < 0 || hops < 1 || E >= lim || G >= lim || int64_t(hops) * N >= lim) return AIMX_HOST_EARG;
  if (!fwd_rowptr || !bwd_rowptr || !graph_rowptr || (E > 0 && (!edges || !fwd_col || !bwd_col)) ||
      (N > 0 && (!batch || !graph_col)))
    return AIMX_HOST_EARG;
  if (E > 0 && N == 0) return AIMX_HOST_EARG;
  const int64_t HN = int64_t(hops) * N;
  for (int64_t i = 0; i < E; ++i)
    if (edges[2 * i] < 0 || edges[2 * i] >= HN) return AIMX_HOST_EARG;
  for (int64_t i = 0; i < N; ++i)
    if (batch[i] < 0 || batch[i] >= G) return AIMX_HOST_EARG;
  try {
    auto src = [&](int64_t i) {
      const int64_t x = edges[2 * i + 1];
      return int32_t(x >= 0 && x < N ? x : ((x % N) + N) % N);
    };
    counting_csr(E, HN, [&](int64_t i) { return edges[2 * i]; }, src, fwd_rowptr, fwd_col);
    counting_csr(E, N, src, [&](int64_t i) { return int32_t(edges[2 * i]); }, bwd_rowptr, bwd_col);
    counting_csr(N, G, [&](int64_t i) { return batch[i]; }, [](int64_t i) { return int32_t(i); }, graph_rowptr,
                 graph_col);
  } catch (const std::bad_alloc&) {
    return AIMX_HOST_ENOMEM;
  }
  return AIMX_HOST_OK;
}

// The same three CSRs for the batch this collator has just written (aimx_collate_write), built by
// its worker pool: a molecule's edges (edge_off[g] .. edge_off[g+1]) join only its own atoms, so
// the rows each worker counts and fills are its molecules' own and the order inside a row (edge
// order) is kept without a global sort. The slack edges past the planned ones (padding self
// loops) are counted and placed on the calling thread, after the molecules' (their order). Input
// that does not have this shape goes to the serial aimx_csr_host_build: identical results.
extern "C" int aimx_collate_csr(aimx_collator* c, const int64_t* edges, int64_t E, const int64_t* batch, int64_t N,
                                int64_t G, int32_t hops, int32_t* fwd_rowptr, int32_t* fwd_col, int32_t* bwd_rowptr,
                                int32_t* bwd_col, int32_t* graph_rowptr, int32_t* graph_col) {
  auto serial = [&] {
    return aimx_csr_host_build(edges, E, batch, N, G, hops, fwd_rowptr, fwd_col, bwd_rowptr, bwd_col, graph_rowptr,
                               graph_col);
  };
  const int64_t lim = int64_t(1) << 31;
  if (!c || !c->planned || E < c->E || N < c->N || G < c->G || E <= 0 || N <= 0 || hops < 1 || E >= lim ||
      G >= lim || int64_t(hops) * N >= lim || !edges || !batch || !fwd_rowptr || !fwd_col || !bwd_rowptr ||
      !bwd_col || !graph_rowptr || !graph_col)
    return serial();
  const int P = c->pool.size();
  const int64_t HN = int64_t(hops) * N, G0 = c->G, N0 = c->N, E0 = c->E;
  try {
    std::atomic<bool> shaped{true};
    // zero the count arrays, check the molecules' locality and batch order, count their rows
    c->pool.run([&](int w) {
      int64_t lo, hi;
      split_range(HN + 1, P, w, &lo, &hi);
      std::fill(fwd_rowptr + lo, fwd_rowptr + hi, 0);
      split_range(N + 1, P, w, &lo, &hi);
      std::fill(bwd_rowptr + lo, bwd_rowptr + hi, 0);
    });
    c->pool.run([&](int w) {
      int64_t lo, hi;
      split_range(N, P, w, &lo, &hi);
      for (int64_t i = lo; i < hi; ++i)
        if (batch[i] < 0 || batch[i] >= G || (i > 0 && batch[i] < batch[i - 1])) {
          shaped = false;
          return;
        }
      split_range(G0, P, w, &lo, &hi);
      for (int64_t g = lo; g < hi; ++g) {
        const int64_t a0 = c->atom_off[g], a1 = c->atom_off[g + 1];
        for (int64_t i = c->edge_off[g]; i < c->edge_off[g + 1]; ++i) {
          const int64_t t = edges[2 * i], u = edges[2 * i + 1];
          if (t < a0 || t >= a1 || u < a0 || u >= a1) {
            shaped = false;
            return;
          }
          ++fwd_rowptr[t + 1];
          ++bwd_rowptr[u + 1];
        }
      }
    });
    if (shaped)
      for (int64_t i = E0; i < E; ++i) {
        const int64_t t = edges[2 * i], u = edges[2 * i + 1];
        if (t < N0 || t >= N || u < N0 || u >= N) {
          shaped = false;
          break;
        }
        ++fwd_rowptr[t + 1];
        ++bwd_rowptr[u + 1];
      }
    if (!shaped) return serial();
    for (int64_t r = 0; r < HN; ++r) fwd_rowptr[r + 1] += fwd_rowptr[r];
    for (int64_t r = 0; r < N; ++r) bwd_rowptr[r + 1] += bwd_rowptr[r];
    c->csr_next_f.assign(fwd_rowptr, fwd_rowptr + N);  // rows >= N (hop offsets) hold no item here
    c->csr_next_b.assign(bwd_rowptr, bwd_rowptr + N);
    int32_t* nf = c->csr_next_f.data();
    int32_t* nb = c->csr_next_b.data();
    c->pool.run([&](int w) {
      int64_t lo, hi;
      split_range(G0, P, w, &lo, &hi);
      for (int64_t i = lo < hi ? c->edge_off[lo] : 0; i < (lo < hi ? c->edge_off[hi] : 0); ++i) {
        const int64_t t = edges[2 * i], u = edges[2 * i + 1];
        fwd_col[nf[t]++] = int32_t(u);
        bwd_col[nb[u]++] = int32_t(t);
      }
    });
    for (int64_t i = E0; i < E; ++i) {
      const int64_t t = edges[2 * i], u = edges[2 * i + 1];
      fwd_col[nf[t]++] = int32_t(u);
      bwd_col[nb[u]++] = int32_t(t);
    }
    // graph CSR: batch is non-decreasing, so the stable order is the identity
    std::fill(graph_rowptr, graph_rowptr + G + 1, 0);
    for (int64_t i = 0; i < N; ++i) ++graph_rowptr[batch[i] + 1];
    for (int64_t g = 0; g < G; ++g) graph_rowptr[g + 1] += graph_rowptr[g];
    for (int64_t i = 0; i < N; ++i) graph_col[i] = int32_t(i);
  } catch (const std::bad_alloc&) {
    return AIMX_HOST_ENOMEM;
  }
  return AIMX_HOST_OK;
}
