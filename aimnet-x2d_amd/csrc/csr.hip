// Stable CSR construction on the device (integer, bit-exact).
//
// The reference never builds a CSR: torch_scatter.scatter_add (layers.py:158-163) runs ATen's CPU
// scatter_add_, which visits edges in ascending edge order per target row. A CSR whose rows keep
// that order lets the hop be a deterministic segmented gather-sum with the reference's exact
// summation order (no float atomics). Pipeline (all on `stream`, no host sync):
//   1. count   : deg[key(i)]++                      (int atomics)
//   2. scan    : rowptr = exclusive_scan(deg)        (3-phase block scan)
//   3. fill    : slot via cursor atomics            (unstable placement, plus key and item id;
//                the cursor is the degree array, re-zeroed by the scan's last phase)
//   4. order   : each item's rank among equal keys = #smaller item ids -> stable final position
#include "aimx_common.h"

namespace aimx {
namespace {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;  // 2048 rows per block

__device__ __forceinline__ int64_t pymod(int64_t v, int64_t m) {
  int64_t r = v % m;
  return r < 0 ? r + m : r;
}

__device__ __forceinline__ int64_t read_key(const int64_t* key, int64_t stride, int64_t mod, int64_t i) {
  int64_t k = key[i * stride];
  return mod > 0 ? pymod(k, mod) : k;
}

__global__ void k_count(const int64_t* __restrict__ key, int64_t stride, int64_t mod, int64_t n_items,
                        int64_t n_rows, int32_t* __restrict__ deg, int32_t* __restrict__ status) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_items;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = read_key(key, stride, mod, i);
    if (k >= 0 && k < n_rows) {
      atomicAdd(&deg[k], 1);
    } else if (status) {
      atomicOr(status, AIMX_STATUS_KEY_OUT_OF_RANGE);
    }
  }
}

// Block-level exclusive scan over kScanTile rows; writes local prefix and the block total.
__global__ __launch_bounds__(kScanThreads) void k_scan_local(const int32_t* __restrict__ in, int64_t n,
                                                             int32_t* __restrict__ out,
                                                             int32_t* __restrict__ block_sums) {
  __shared__ int32_t wsum[kScanThreads / kWave];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int32_t v[kScanItems];
  int32_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = (base + j < n) ? in[base + j] : 0;
    s += v[j];
  }
  // inclusive wave scan of per-thread sums
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  int32_t incl = s;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    int32_t t = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += t;
  }
  if (lane == kWave - 1) wsum[wid] = incl;
  __syncthreads();
  int32_t woff = 0;
  for (int w = 0; w < wid; ++w) woff += wsum[w];
  int32_t run = woff + incl - s;  // exclusive prefix of this thread
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
  if (threadIdx.x == kScanThreads - 1) block_sums[blockIdx.x] = woff + incl;
}

// Single workgroup: exclusive scan of the block sums in place; total -> *total.
__global__ __launch_bounds__(1024) void k_scan_sums(int32_t* __restrict__ sums, int64_t nb, int32_t* __restrict__ total) {
  __shared__ int32_t wsum[1024 / kWave];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int32_t s = i < nb ? sums[i] : 0;
    int32_t incl = s;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      int32_t t = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += t;
    }
    if (lane == kWave - 1) wsum[wid] = incl;
    __syncthreads();
    int32_t woff = 0;
    for (int w = 0; w < wid; ++w) woff += wsum[w];
    const int32_t c = carry;
    if (i < nb) sums[i] = c + woff + incl - s;
    __syncthreads();
    if (threadIdx.x == 1023) carry = c + woff + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// Adds the block offsets and re-zeroes the degree array, which k_fill then uses as the per-row
// insertion cursor (no separate memset: runtime memset nodes are avoided in captured graphs).
__global__ __launch_bounds__(kScanThreads) void k_scan_add(int32_t* __restrict__ out, int64_t n,
                                                           const int32_t* __restrict__ block_offs,
                                                           int32_t* __restrict__ deg) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  const int32_t off = block_offs[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kScanItems; ++j)
    if (base + j < n) {
      out[base + j] += off;
      deg[base + j] = 0;
    }
}

__global__ void k_zero_i32(int32_t* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0;
}

// p[0..n) = 0 and, when q is non-null, *q = 0 (the multi build's status word) in the same launch
__global__ void k_zero_i32_and(int32_t* __restrict__ p, int64_t n, int32_t* __restrict__ q) {
  if (q && blockIdx.x == 0 && threadIdx.x == 0) *q = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0;
}

__global__ void k_fill(const int64_t* __restrict__ key, int64_t kstride, int64_t kmod,
                       const int64_t* __restrict__ val, int64_t vstride, int64_t vmod, int64_t n_items,
                       int64_t n_rows, const int32_t* __restrict__ rowptr, int32_t* __restrict__ cursor,
                       int32_t* __restrict__ t_key, int32_t* __restrict__ t_val, int32_t* __restrict__ t_id) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_items;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = read_key(key, kstride, kmod, i);
    if (k < 0 || k >= n_rows) continue;
    const int32_t pos = rowptr[k] + atomicAdd(&cursor[k], 1);
    int64_t v = i;
    if (val) {
      v = val[i * vstride];
      if (vmod > 0) v = pymod(v, vmod);
    }
    t_key[pos] = (int32_t)k;
    t_val[pos] = (int32_t)v;
    t_id[pos] = (int32_t)i;
  }
}

__global__ void k_order(int64_t n_valid_max, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ total,
                        const int32_t* __restrict__ t_key, const int32_t* __restrict__ t_val,
                        const int32_t* __restrict__ t_id, int32_t* __restrict__ col) {
  const int32_t n_valid = *total;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n_valid_max && p < n_valid;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = t_key[p];
    const int32_t b = rowptr[k], e = rowptr[k + 1];
    const int32_t me = t_id[p];
    int32_t rank = 0;
    for (int32_t q = b; q < e; ++q) rank += (t_id[q] < me) ? 1 : 0;
    col[b + rank] = t_val[p];
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" size_t aimx_csr_workspace_bytes(int64_t n_items, int64_t n_rows) {
  const int64_t nb = cdiv(n_rows > 0 ? n_rows : 1, kScanTile);
  return align256(sizeof(int32_t) * (size_t)(n_rows + 1)) +      // deg / cursor
         align256(sizeof(int32_t) * (size_t)(nb + 1)) +          // block sums (+ total)
         3 * align256(sizeof(int32_t) * (size_t)(n_items + 1));  // t_key, t_val, t_id
}

extern "C" int aimx_csr_build(const int64_t* key, int64_t key_stride, int64_t key_mod, const int64_t* val,
                              int64_t val_stride, int64_t val_mod, int64_t n_items, int64_t n_rows, int32_t* rowptr,
                              int32_t* col, void* workspace, size_t workspace_bytes, int32_t* status,
                              aimx_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (n_items < 0 || n_rows < 0 || n_items > INT32_MAX || n_rows >= INT32_MAX) return AIMX_EARG;
  if (!rowptr || (n_items > 0 && (!key || !col))) return AIMX_EARG;
  if (workspace_bytes < aimx_csr_workspace_bytes(n_items, n_rows) || !workspace) return AIMX_EARG;
  const int64_t nb = cdiv(n_rows > 0 ? n_rows : 1, kScanTile);
  char* ws = (char*)workspace;
  int32_t* deg = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(n_rows + 1));
  int32_t* bsum = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(nb + 1));
  int32_t* t_key = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(n_items + 1));
  int32_t* t_val = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(n_items + 1));
  int32_t* t_id = (int32_t*)ws;

  const int threads = 256;
  // zero-fill by kernel: hipMemsetAsync nodes misbehaved on graph replay (ROCm 7.2)
  hipLaunchKernelGGL(k_zero_i32, dim3((unsigned)std::min<int64_t>(cdiv(n_rows + 1, threads), 4096)), dim3(threads),
                     0, stream, deg, n_rows + 1);
  AIMX_CHECK_LAUNCH();
  const int64_t grid_items = std::min<int64_t>(cdiv(n_items > 0 ? n_items : 1, threads), 8192);
  if (n_items > 0) {
    hipLaunchKernelGGL(k_count, dim3((unsigned)grid_items), dim3(threads), 0, stream, key, key_stride, key_mod,
                       n_items, n_rows, deg, status);
    AIMX_CHECK_LAUNCH();
  }
  // rowptr[0..n_rows) = exclusive scan(deg); rowptr[n_rows] = total
  if (n_rows > 0) {
    hipLaunchKernelGGL(k_scan_local, dim3((unsigned)nb), dim3(kScanThreads), 0, stream, deg, n_rows, rowptr, bsum);
    AIMX_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, stream, bsum, nb, rowptr + n_rows);
    AIMX_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(kScanThreads), 0, stream, rowptr, n_rows, bsum, deg);
    AIMX_CHECK_LAUNCH();
  } else {
    hipLaunchKernelGGL(k_zero_i32, dim3(1), dim3(64), 0, stream, rowptr, (int64_t)1);
    AIMX_CHECK_LAUNCH();
  }
  if (n_items == 0 || n_rows == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)grid_items), dim3(threads), 0, stream, key, key_stride, key_mod, val,
                     val_stride, val_mod, n_items, n_rows, rowptr, deg, t_key, t_val, t_id);
  AIMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_order, dim3((unsigned)grid_items), dim3(threads), 0, stream, n_items, rowptr,
                     rowptr + n_rows, t_key, t_val, t_id, col);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

// ---------------------------------------------------------------------------------------------
// Several CSRs in one pass (the plan's fwd / bwd / graph CSRs): one launch per phase for all of
// them. Rows of all specs are concatenated (spec s owns global rows [row0_s, row0_s + rows_s)),
// items likewise; one scan over all rows gives global positions, and each spec's rowptr is the
// scan relative to its first row.
// ---------------------------------------------------------------------------------------------
namespace aimx {
namespace {

constexpr int kMaxSpecs = 4;
struct MultiTable {
  int32_t n;
  int64_t item0[kMaxSpecs + 1], row0[kMaxSpecs + 1];
  AimxCsrSpec s[kMaxSpecs];
};

__device__ __forceinline__ int spec_of_item(const MultiTable& t, int64_t i) {
  int q = 0;
  while (q + 1 < t.n && t.item0[q + 1] <= i) ++q;
  return q;
}
__device__ __forceinline__ int spec_of_row(const MultiTable& t, int64_t r) {
  int q = 0;
  while (q + 1 < t.n && t.row0[q + 1] <= r) ++q;
  return q;
}

__global__ void k_count_multi(const MultiTable t, int32_t* __restrict__ deg, int32_t* __restrict__ status) {
  const int64_t total = t.item0[t.n];
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int q = spec_of_item(t, g);
    const AimxCsrSpec& sp = t.s[q];
    const int64_t k = read_key(sp.key, sp.key_stride, sp.key_mod, g - t.item0[q]);
    if (k >= 0 && k < sp.n_rows) {
      atomicAdd(&deg[t.row0[q] + k], 1);
    } else if (status) {
      atomicOr(status, AIMX_STATUS_KEY_OUT_OF_RANGE);
    }
  }
}

__global__ void k_fill_multi(const MultiTable t, const int32_t* __restrict__ scan, int32_t* __restrict__ cursor,
                             int32_t* __restrict__ t_key, int32_t* __restrict__ t_val, int32_t* __restrict__ t_id) {
  const int64_t total = t.item0[t.n];
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int q = spec_of_item(t, g);
    const AimxCsrSpec& sp = t.s[q];
    const int64_t i = g - t.item0[q];
    const int64_t k = read_key(sp.key, sp.key_stride, sp.key_mod, i);
    if (k < 0 || k >= sp.n_rows) continue;
    const int64_t row = t.row0[q] + k;
    const int32_t pos = scan[row] + atomicAdd(&cursor[row], 1);
    int64_t v = i;
    if (sp.val) {
      v = sp.val[i * sp.val_stride];
      if (sp.val_mod > 0) v = pymod(v, sp.val_mod);
    }
    t_key[pos] = (int32_t)row;
    t_val[pos] = (int32_t)v;
    t_id[pos] = (int32_t)i;
  }
}

// Threads over max(valid items, rows + specs): stable placement of every item, and each spec's
// rowptr = global scan relative to the spec's first row.
__global__ void k_order_multi(const MultiTable t, int64_t work, const int32_t* __restrict__ scan,
                              const int32_t* __restrict__ t_key, const int32_t* __restrict__ t_val,
                              const int32_t* __restrict__ t_id) {
  const int64_t R = t.row0[t.n];
  const int32_t n_valid = scan[R];
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < work; g += (int64_t)gridDim.x * blockDim.x) {
    if (g < n_valid) {
      const int32_t row = t_key[g];
      const int q = spec_of_row(t, row);
      const int32_t b = scan[row], e = scan[row + 1];
      const int32_t me = t_id[g];
      int32_t rank = 0;
      for (int32_t p = b; p < e; ++p) rank += (t_id[p] < me) ? 1 : 0;
      t.s[q].col[b - scan[t.row0[q]] + rank] = t_val[g];
    }
    // rowptr entries: global row index r in [0, R + n) -> spec q, local i in [0, rows_q]
    if (g < R + t.n) {
      int q = 0;
      while (q + 1 < t.n && g >= t.row0[q + 1] + (q + 1)) ++q;
      const int64_t i = g - t.row0[q] - q;
      if (i <= t.s[q].n_rows) t.s[q].rowptr[i] = scan[t.row0[q] + i] - scan[t.row0[q]];
    }
  }
}

}  // namespace
}  // namespace aimx

extern "C" size_t aimx_csr_build_multi_workspace_bytes(const AimxCsrSpec* specs, int32_t n) {
  if (!specs || n < 1 || n > aimx::kMaxSpecs) return 0;
  int64_t R = 0, I = 0;
  for (int32_t i = 0; i < n; ++i) R += specs[i].n_rows, I += specs[i].n_items;
  const int64_t nb = cdiv(R > 0 ? R : 1, aimx::kScanTile);
  return 2 * aimx::align256(sizeof(int32_t) * (size_t)(R + 1)) + aimx::align256(sizeof(int32_t) * (size_t)(nb + 1)) +
         3 * aimx::align256(sizeof(int32_t) * (size_t)(I + 1));
}

extern "C" int aimx_csr_build_multi(const AimxCsrSpec* specs, int32_t n, void* workspace, size_t workspace_bytes,
                                    int32_t* status, aimx_stream_t stream_) {
  using namespace aimx;
  hipStream_t stream = (hipStream_t)stream_;
  if (!specs || n < 1 || n > kMaxSpecs) return AIMX_EARG;
  MultiTable t{};
  t.n = n;
  int64_t R = 0, I = 0;
  for (int32_t i = 0; i < n; ++i) {
    const AimxCsrSpec& sp = specs[i];
    if (sp.n_items < 0 || sp.n_rows < 0 || !sp.rowptr || (sp.n_items > 0 && (!sp.key || !sp.col))) return AIMX_EARG;
    t.s[i] = sp;
    t.item0[i] = I;
    t.row0[i] = R;
    I += sp.n_items;
    R += sp.n_rows;
  }
  t.item0[n] = I;
  t.row0[n] = R;
  if (I > INT32_MAX || R >= INT32_MAX) return AIMX_EARG;
  if (!workspace || workspace_bytes < aimx_csr_build_multi_workspace_bytes(specs, n)) return AIMX_EARG;
  const int64_t nb = cdiv(R > 0 ? R : 1, kScanTile);
  char* ws = (char*)workspace;
  int32_t* deg = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(R + 1));
  int32_t* scan = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(R + 1));
  int32_t* bsum = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(nb + 1));
  int32_t* t_key = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(I + 1));
  int32_t* t_val = (int32_t*)ws;
  ws += align256(sizeof(int32_t) * (size_t)(I + 1));
  int32_t* t_id = (int32_t*)ws;
  const int threads = 256;
  hipLaunchKernelGGL(k_zero_i32_and, dim3((unsigned)std::min<int64_t>(cdiv(R + 1, threads), 4096)), dim3(threads), 0,
                     stream, deg, R + 1, status);
  AIMX_CHECK_LAUNCH();
  const int64_t grid_items = std::min<int64_t>(cdiv(I > 0 ? I : 1, threads), 8192);
  if (I > 0) {
    hipLaunchKernelGGL(k_count_multi, dim3((unsigned)grid_items), dim3(threads), 0, stream, t, deg, status);
    AIMX_CHECK_LAUNCH();
  }
  // scan[0..R) = exclusive scan(deg); scan[R] = total; deg re-zeroed (the fill cursor)
  if (R > 0) {
    hipLaunchKernelGGL(k_scan_local, dim3((unsigned)nb), dim3(kScanThreads), 0, stream, deg, R, scan, bsum);
    AIMX_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, stream, bsum, nb, scan + R);
    AIMX_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(kScanThreads), 0, stream, scan, R, bsum, deg);
    AIMX_CHECK_LAUNCH();
  } else {
    hipLaunchKernelGGL(k_zero_i32, dim3(1), dim3(64), 0, stream, scan, (int64_t)1);
    AIMX_CHECK_LAUNCH();
  }
  if (I > 0) {
    hipLaunchKernelGGL(k_fill_multi, dim3((unsigned)grid_items), dim3(threads), 0, stream, t, (const int32_t*)scan, deg,
                       t_key, t_val, t_id);
    AIMX_CHECK_LAUNCH();
  }
  const int64_t work = std::max<int64_t>(I, R + n);
  hipLaunchKernelGGL(k_order_multi, dim3((unsigned)std::min<int64_t>(cdiv(work, threads), 8192)), dim3(threads), 0,
                     stream, t, work, (const int32_t*)scan, t_key, t_val, t_id);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
