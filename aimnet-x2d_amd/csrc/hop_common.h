// Helpers shared by the two hop kernels (hop.hip: 16-byte-aligned rows; hop_unal.hip: any row
// alignment / odd widths). Reference op: ShellConvolutionLayer.message_passing,
// src/models/layers.py:133-167.
#pragma once

#include <stdint.h>

#include "aimx_common.h"

namespace aimx {

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

// The odd-width / unaligned-row hop by 16-byte vectors at 4-byte-aligned addresses (hop_unal.hip);
// same contract as aimx_segment_gather_sum.
int launch_gather_unal(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out, int64_t out_ld,
                       int64_t out_rpc, int64_t out_cs, const float* add0, int64_t add0_ld, const float* add1,
                       int64_t add1_ld, const int64_t* row_seg, int64_t row_seg_stride, hipStream_t stream,
                       int32_t skip_tail);

}  // namespace aimx
