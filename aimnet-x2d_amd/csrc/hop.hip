// The hop: segmented gather-sum over a stable CSR (HBM-bound integer-indexed row traffic).
//
// Reference: ShellConvolutionLayer.message_passing, src/models/layers.py:133-167
//   aggregated = scatter_add(x[src % N], target, dim_size = num_hops * N)
// Here each output row t is produced by ONE owner (no atomics): it walks its CSR segment
// (edges with target t, ascending edge id) and sums the source rows in that order starting from
// +0.0f, which reproduces CPU ATen scatter_add_ bit for bit. Lanes run along the feature dim with
// VEC-wide (16/8/4-byte) loads; a 64-lane wave covers 64*VEC consecutive floats of the flattened
// [rows, D] output, so the stores and the gathered source rows are coalesced, and the index loads
// (rowptr/col, int32) are broadcast within a row. Source rows of one molecule sit together in
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

template <int VEC>
__global__ __launch_bounds__(256) void k_gather_sum(const float* __restrict__ src, int64_t src_ld, FastDiv src_rpc,
                                                     int64_t src_cs, FastDiv units_per_row,
                                                     const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col, uint32_t rows,
                                                     float* __restrict__ out, int64_t out_ld, FastDiv out_rpc,
                                                     int64_t out_cs, const float* __restrict__ add0, int64_t add0_ld,
                                                     const float* __restrict__ add1, int64_t add1_ld) {
  using T = typename VecT<VEC>::T;
  const uint32_t total = rows * units_per_row.d;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const uint32_t r = fdiv(t, units_per_row);
    const uint32_t u = (t - r * units_per_row.d) * VEC;
    const int32_t b = rowptr[r], e = rowptr[r + 1];
    T acc = vzero<T>();
    int32_t k = b;
    // 4 independent gathers in flight, summed in edge order.
    for (; k + 4 <= e; k += 4) {
      const int32_t c0 = col[k], c1 = col[k + 1], c2 = col[k + 2], c3 = col[k + 3];
      const T v0 = *reinterpret_cast<const T*>(src + row_off(c0, src_ld, src_rpc, src_cs) + u);
      const T v1 = *reinterpret_cast<const T*>(src + row_off(c1, src_ld, src_rpc, src_cs) + u);
      const T v2 = *reinterpret_cast<const T*>(src + row_off(c2, src_ld, src_rpc, src_cs) + u);
      const T v3 = *reinterpret_cast<const T*>(src + row_off(c3, src_ld, src_rpc, src_cs) + u);
      vadd(acc, v0);
      vadd(acc, v1);
      vadd(acc, v2);
      vadd(acc, v3);
    }
    for (; k < e; ++k) {
      const int32_t c0 = col[k];
      vadd(acc, *reinterpret_cast<const T*>(src + row_off(c0, src_ld, src_rpc, src_cs) + u));
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
  const int64_t blocks = std::min<int64_t>(cdiv(rows * upr_i, threads), 256 * 32);
  if (vec == 4)
    hipLaunchKernelGGL(k_gather_sum<4>, dim3((unsigned)blocks), dim3(threads), 0, stream, src, src_ld, srpc,
                       src_cs, upr, rowptr, col, (uint32_t)rows, out, out_ld, orpc, out_cs, add0, add0_ld, add1, add1_ld);
  else if (vec == 2)
    hipLaunchKernelGGL(k_gather_sum<2>, dim3((unsigned)blocks), dim3(threads), 0, stream, src, src_ld, srpc,
                       src_cs, upr, rowptr, col, (uint32_t)rows, out, out_ld, orpc, out_cs, add0, add0_ld, add1, add1_ld);
  else
    hipLaunchKernelGGL(k_gather_sum<1>, dim3((unsigned)blocks), dim3(threads), 0, stream, src, src_ld, srpc,
                       src_cs, upr, rowptr, col, (uint32_t)rows, out, out_ld, orpc, out_cs, add0, add0_ld, add1, add1_ld);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
