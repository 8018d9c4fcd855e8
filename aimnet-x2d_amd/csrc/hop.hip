// The hop: segmented gather-sum over a stable CSR (HBM-bound integer-indexed row traffic).
//
// Reference: ShellConvolutionLayer.message_passing, src/models/layers.py:133-167
//   aggregated = scatter_add(x[src % N], target, dim_size = num_hops * N)
// Here each output row t is produced by ONE owner (no atomics): it walks its CSR segment
// (edges with target t, ascending edge id) and sums the source rows in that order starting from
// +0.0f, which reproduces CPU ATen scatter_add_ bit for bit. Lanes run along the feature dim with
// VEC-wide (16/8/4-byte) loads; a 64-lane wave covers 64*VEC consecutive floats of the flattened
// [rows, D] output, so the stores and the gathered source rows are coalesced. A workgroup owns a
// tile of consecutive rows and stages the tile's rowptr/col slices in LDS first (see k_gather_sum
// below). Source rows of one molecule sit together in
// HBM, so neighbour re-reads hit L2; the only compulsory HBM traffic is x once, the CSR once and
// the output once (SURVEY.md §8d algorithmic bytes).
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

template <int VEC>
struct VecT;
template <>
struct VecT<1> {
  using T = float;
};
template <>
struct VecT<2> {
  using T = float2;
};
template <>
struct VecT<4> {
  using T = float4;
};

__device__ __forceinline__ void vadd(float& a, const float& b) { a += b; }
__device__ __forceinline__ void vadd(float2& a, const float2& b) {
  a.x += b.x;
  a.y += b.y;
}
__device__ __forceinline__ void vadd(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}
template <typename T>
__device__ __forceinline__ T vzero();
template <>
__device__ __forceinline__ float vzero<float>() { return 0.f; }
template <>
__device__ __forceinline__ float2 vzero<float2>() { return make_float2(0.f, 0.f); }
template <>
__device__ __forceinline__ float4 vzero<float4>() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// Division by a run-time invariant (Granlund-Montgomery), valid for n < 2^31.
struct FastDiv {
  uint32_t d, m, l;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{d, 0, 0};
  if (d == 0) return f;
  while ((1ull << f.l) < d) ++f.l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << f.l) - d)) / d) + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(f.m, n) + n) >> f.l; }

// Row r of a chunked matrix: base + (r % rpc)*ld + (r / rpc)*chunk_stride (rpc == 0: plain rows).
__device__ __forceinline__ int64_t row_off(uint32_t r, int64_t ld, const FastDiv& rpc, int64_t cstride) {
  if (rpc.d == 0) return (int64_t)r * ld;
  const uint32_t q = fdiv(r, rpc);
  return (int64_t)(r - q * rpc.d) * ld + (int64_t)q * cstride;
}

// Row tiles: a workgroup owns `tile_rows` consecutive output rows. It stages their rowptr slice and
// (when it fits) their whole col slice in LDS with two coalesced loads, so the per-output-element
// dependency chain is LDS -> gathered source row -> store instead of rowptr -> col -> row in HBM.
// A tile whose rows hold no edges (the reference's hop chunks >= 1 are all-empty, layers.py:154)
// becomes a pure streaming store. Gathers are issued 8 at a time with clamped (always valid)
// indices and summed with selects, so the sum is the ordered edge-order sum bit for bit.
constexpr int kMaxTileRows = 64;
constexpr int kColCap = 4096;  // staged col entries per tile (16 KiB)
constexpr int kGroup = 8;      // gathers in flight per thread

template <bool CHUNKED>
__device__ __forceinline__ int64_t src_off(uint32_t c, int64_t ld, const FastDiv& rpc, int64_t cs) {
  if (!CHUNKED) return (int64_t)c * ld;
  const uint32_t q = fdiv(c, rpc);
  return (int64_t)(c - q * rpc.d) * ld + (int64_t)q * cs;
}

template <int VEC, bool LDS_COL, bool SRC_CHUNKED>
__device__ __forceinline__ void tile_body(const float* __restrict__ src, int64_t src_ld, const FastDiv& src_rpc,
                                          int64_t src_cs, const FastDiv& upr, const int32_t* s_ptr,
                                          const int32_t* cols, int32_t base, uint32_t r0, uint32_t nr,
                                          float* __restrict__ out, int64_t out_ld, const FastDiv& out_rpc,
                                          int64_t out_cs, const float* __restrict__ add0, int64_t add0_ld,
                                          const float* __restrict__ add1, int64_t add1_ld, bool any_edges) {
  using T = typename VecT<VEC>::T;
  const uint32_t units = nr * upr.d;
  for (uint32_t t = threadIdx.x; t < units; t += blockDim.x) {
    const uint32_t rl = fdiv(t, upr);
    const uint32_t u = (t - rl * upr.d) * VEC;
    const uint32_t r = r0 + rl;
    T acc = vzero<T>();
    if (any_edges) {
      const int32_t b = s_ptr[rl] - (LDS_COL ? base : 0), e = s_ptr[rl + 1] - (LDS_COL ? base : 0);
      for (int32_t k = b; k < e; k += kGroup) {
        T v[kGroup];
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
          const int32_t c = cols[min(k + j, e - 1)];
          v[j] = *reinterpret_cast<const T*>(src + src_off<SRC_CHUNKED>((uint32_t)c, src_ld, src_rpc, src_cs) + u);
        }
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
          T s = acc;
          vadd(s, v[j]);
          if (k + j < e) acc = s;
        }
      }
    }
    if (add0) {
      T s = *reinterpret_cast<const T*>(add0 + (int64_t)r * add0_ld + u);
      vadd(s, acc);
      acc = s;
    }
    if (add1) vadd(acc, *reinterpret_cast<const T*>(add1 + (int64_t)r * add1_ld + u));
    *reinterpret_cast<T*>(out + row_off(r, out_ld, out_rpc, out_cs) + u) = acc;
  }
}

template <int VEC, bool SRC_CHUNKED>
__global__ __launch_bounds__(256) void k_gather_sum(const float* __restrict__ src, int64_t src_ld, FastDiv src_rpc,
                                                     int64_t src_cs, FastDiv upr, const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col, uint32_t rows, uint32_t tile_rows,
                                                     float* __restrict__ out, int64_t out_ld, FastDiv out_rpc,
                                                     int64_t out_cs, const float* __restrict__ add0, int64_t add0_ld,
                                                     const float* __restrict__ add1, int64_t add1_ld) {
  __shared__ int32_t s_ptr[kMaxTileRows + 1];
  __shared__ int32_t s_col[kColCap];
  const uint32_t r0 = blockIdx.x * tile_rows;
  const uint32_t nr = min(tile_rows, rows - r0);
  if (threadIdx.x <= nr) s_ptr[threadIdx.x] = rowptr[r0 + threadIdx.x];
  __syncthreads();
  const int32_t base = s_ptr[0];
  const int32_t ncols = s_ptr[nr] - base;
  if (ncols <= kColCap) {
    for (int32_t i = threadIdx.x; i < ncols; i += blockDim.x) s_col[i] = col[base + i];
    __syncthreads();
    tile_body<VEC, true, SRC_CHUNKED>(src, src_ld, src_rpc, src_cs, upr, s_ptr, s_col, base, r0, nr, out, out_ld, out_rpc, out_cs,
                         add0, add0_ld, add1, add1_ld, ncols > 0);
  } else {
    tile_body<VEC, false, SRC_CHUNKED>(src, src_ld, src_rpc, src_cs, upr, s_ptr, col, base, r0, nr, out, out_ld, out_rpc, out_cs,
                          add0, add0_ld, add1, add1_ld, true);
  }
}

inline bool aligned(const void* p, int bytes) { return ((uintptr_t)p % bytes) == 0; }

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" int aimx_segment_gather_sum(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out,
                                       int64_t out_ld, int64_t out_rpc, int64_t out_cs, const float* add0,
                                       int64_t add0_ld, const float* add1, int64_t add1_ld, aimx_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (rows < 0 || D < 0) return AIMX_EARG;
  if (rows == 0 || D == 0) return AIMX_OK;
  if (!src || !rowptr || !out) return AIMX_EARG;
  auto ok = [&](int v) {
    const int b = 4 * v;
    if (D % v || src_ld % v || out_ld % v || src_cs % v || out_cs % v) return false;
    if (!aligned(src, b) || !aligned(out, b)) return false;
    if (add0 && (add0_ld % v || !aligned(add0, b))) return false;
    if (add1 && (add1_ld % v || !aligned(add1, b))) return false;
    return true;
  };
  const int vec = ok(4) ? 4 : (ok(2) ? 2 : 1);
  const int64_t upr_i = D / vec;
  // 32-bit thread indexing (rows * D / vec < 2^31) and int32 chunked row ids.
  if (rows * upr_i >= (int64_t)INT32_MAX || src_rpc >= INT32_MAX || out_rpc >= INT32_MAX) return AIMX_EARG;
  const FastDiv upr = make_fastdiv((uint32_t)upr_i);
  const FastDiv srpc = make_fastdiv(src_rpc > 0 ? (uint32_t)src_rpc : 0);
  const FastDiv orpc = make_fastdiv(out_rpc > 0 ? (uint32_t)out_rpc : 0);
  const int threads = 256;
  // tile height: ~2 vector units per thread, then shorter tiles while the grid is under 4
  // workgroups per CU (small batches are latency-bound: more workgroups hide more latency)
  int64_t tr = std::min<int64_t>(kMaxTileRows, std::max<int64_t>(1, 2 * threads / upr_i));
  while (tr > 1 && cdiv(rows, tr) < 1024) tr = std::max<int64_t>(1, tr / 2);
  const int64_t blocks = cdiv(rows, tr);
  using KFn = void (*)(const float*, int64_t, FastDiv, int64_t, FastDiv, const int32_t*, const int32_t*, uint32_t,
                      uint32_t, float*, int64_t, FastDiv, int64_t, const float*, int64_t, const float*, int64_t);
  const bool chunked = src_rpc > 0;
  KFn fn = vec == 4 ? (chunked ? k_gather_sum<4, true> : k_gather_sum<4, false>)
           : vec == 2 ? (chunked ? k_gather_sum<2, true> : k_gather_sum<2, false>)
                      : (chunked ? k_gather_sum<1, true> : k_gather_sum<1, false>);
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(threads), 0, stream, src, src_ld, srpc, src_cs, upr, rowptr, col,
                     (uint32_t)rows, (uint32_t)tr, out, out_ld, orpc, out_cs, add0, add0_ld, add1, add1_ld);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
