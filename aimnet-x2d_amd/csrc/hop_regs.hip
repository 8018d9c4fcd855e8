// The hop's molecule rows summed from the register file (round 5). Same contract and bit-exact
// result as hop.hip / hop_rows.hip (the ordered edge-order sum of CPU scatter_add_, reference
// src/models/layers.py:133-167, and its backward); used for the rows that are not runs of 16-byte
// vectors (odd D = 153 / 307, unaligned hop chunks), where hop_rows.hip's LDS design spends most of
// its time in dependent phases (stage -> barrier -> sum -> barrier -> realign -> barrier -> store per
// 80-column pass: c4's backward ran at 2.4 TB/s, c5's at 2.0 with its LDS read rate as the bound).
//
// A wave owns one window of kGW rows of the first output chunk and one 64-column block: for every
// molecule that STARTS in the window (molecule ids from row_seg, one ballot per 64 rows), lane l
// loads column c0 + l of the molecule's first 64 source rows into two 32-register vectors (all the
// loads in flight at once, dword accesses: any row alignment is free), then walks the molecule's
// output rows: each CSR segment is summed in edge order (its source indices are wave-uniform: scalar
// loads) by reading the source's register with a wave-uniform index (s_set_gpr_idx) — no LDS, no
// barrier, no realignment; a source outside the molecule's register block (general inputs: hop-offset
// targets, molecules > 64 atoms, edges across molecules) is loaded from memory instead. The sums are
// the same sequential fp32 adds in the same order, so the result is bit-identical to the other
// kernels; the residual terms of the backward are added as they do (add0 + sum, then + add1).
// Output rows past the first chunk (hop chunks >= 1: zero fills, or general targets) stay with
// hop_rows.hip's big tiles (launched with no windows).
#include <algorithm>
#include <cstdlib>

#include "aimx_common.h"
#include "hop_common.h"

namespace aimx {
namespace {

constexpr int kGW = 64;       // window rows per wave
constexpr int kColLds = 1536;  // col entries of a molecule staged in LDS (6 KiB per wave)
typedef float vreg32 __attribute__((ext_vector_type(32)));

struct RegsArgs {
  const float* src;
  int64_t src_ld, src_cs;
  FastDiv src_rpc;
  const int32_t* rowptr;
  const int32_t* col;
  uint32_t D, ncb, split;  // width, 64-column blocks, rows of the first output chunk
  float* out;
  int64_t out_ld;
  const float* add0;
  int64_t add0_ld;
  const float* add1;
  int64_t add1_ld;
  const int64_t* seg;
  int64_t seg_stride;
};

template <bool SRC_CHUNKED>
__device__ __forceinline__ const float* src_row(const RegsArgs& a, uint32_t q) {
  if (!SRC_CHUNKED) return a.src + (int64_t)q * a.src_ld;
  const uint32_t k = fdiv(q, a.src_rpc);
  return a.src + (int64_t)(q - k * a.src_rpc.d) * a.src_ld + (int64_t)k * a.src_cs;
}

// molecule-start bits of rows [base, base + 64) (rows >= split never start one)
__device__ __forceinline__ uint64_t start_bits(const RegsArgs& a, uint32_t base) {
  const uint32_t r = base + (threadIdx.x & 63);
  bool st = false;
  if (r < a.split) st = r == 0 || a.seg[(int64_t)r * a.seg_stride] != a.seg[(int64_t)(r - 1) * a.seg_stride];
  return __ballot(st);
}

// register rel (< 64, wave-uniform) of the molecule's block. The branches are wave-uniform (SALU);
// the empty asm keeps hipcc from if-converting them into a select of both whole vectors.
__device__ __forceinline__ float reg_at(const vreg32& xa, const vreg32& xb, int rel) {
  float v;
  if (rel < 32) {
    v = xa[rel];
    __asm__ volatile("" ::"v"(v));
  } else {
    v = xb[rel - 32];
    __asm__ volatile("" ::"v"(v));
  }
  return v;
}

template <bool SRC_CHUNKED>
__device__ __forceinline__ float from_src(const RegsArgs& a, const vreg32& xa, const vreg32& xb, int32_t q,
                                          uint32_t ms, uint32_t nr, uint32_t c, bool cv) {
  const int32_t rel = q - (int32_t)ms;
  float v;
  if ((uint32_t)rel < nr) {
    v = reg_at(xa, xb, rel);
  } else {  // outside the molecule's register block: from memory (general inputs)
    v = cv ? src_row<SRC_CHUNKED>(a, (uint32_t)q)[c] : 0.f;
  }
  return v;
}

template <bool SRC_CHUNKED>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void k_gather_regs(const RegsArgs a) {
  // the molecule's col slice, staged once per molecule (wave-private: this workgroup is one wave)
  __shared__ int32_t s_col[kColLds];
  const int lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x / a.ncb, cb = blockIdx.x - w * a.ncb;
  const uint32_t R0 = w * kGW, R1 = min(R0 + (uint32_t)kGW, a.split);
  const uint32_t c = cb * 64 + lane;
  const bool cv = c < a.D;
  const uint64_t bits = start_bits(a, R0);
  // first molecule that starts in [R0, R1)
  const uint64_t own = (R1 - R0) >= 64 ? ~0ull : ((1ull << (R1 - R0)) - 1);
  if (!(bits & own)) return;
  uint32_t ms = R0 + (uint32_t)__builtin_ctzll(bits & own);
  while (ms < R1) {
    // its end: the next start after ms (scanning on past this block if needed)
    uint32_t me = a.split;
    {
      const uint64_t rest = (ms - R0 + 1 < 64) ? (bits >> (ms - R0 + 1)) : 0ull;
      if (rest) {
        me = ms + 1 + (uint32_t)__builtin_ctzll(rest);
      } else {
        for (uint32_t b2 = R0 + 64; b2 < a.split; b2 += 64) {
          const uint64_t m2 = start_bits(a, b2);
          if (m2) {
            me = b2 + (uint32_t)__builtin_ctzll(m2);
            break;
          }
        }
      }
    }
    const uint32_t n = me - ms, nr = min(n, 64u);
    // 1) every load in flight at once: the molecule's first 64 source rows (column c), its row
    //    pointers, its col slice (into LDS)
    const float* s0 = src_row<SRC_CHUNKED>(a, ms);  // chunk 0: rows ms.. are consecutive
    const uint32_t bytes = 4u * (uint32_t)((int64_t)(nr - 1) * a.src_ld + a.D);
    const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(s0, bytes);
    // offset = lane part (4c, or 2^30 past the extent for c >= D) + row part (wave-uniform, 2^31 for
    // rows >= nr): no sum wraps (extent < 2^29, checked at launch). The opaque zero keeps hipcc from
    // hoisting the 64 loop-invariant row offsets out of the molecule loop into 64 live VGPRs.
    uint32_t zero;
    __asm__ volatile("s_mov_b32 %0, 0" : "=s"(zero));
    const uint32_t vlane = cv ? 4u * c : 0x40000000u;
    const uint32_t rstep = 4u * (uint32_t)a.src_ld;
    vreg32 xa, xb;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
      const uint32_t ra = ((uint32_t)r < nr ? (uint32_t)r * rstep : 0x80000000u) + zero;
      const uint32_t rb = ((uint32_t)r + 32 < nr ? (uint32_t)(r + 32) * rstep : 0x80000000u) + zero;
      xa[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vlane + ra, 0, 0));
      xb[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vlane + rb, 0, 0));
    }
    // row pointers: lane i holds rowptr[ms + i] (n + 1 <= 65 of them in two loads)
    const int32_t rp_lo = a.rowptr[min(ms + (uint32_t)lane, me)];
    const int32_t rp_hi = a.rowptr[min(ms + 64u + (uint32_t)lane, me)];
    const int32_t b0 = a.rowptr[ms], e0 = a.rowptr[me];  // (scalar)
    const int32_t len = e0 - b0;
    const bool staged = len <= kColLds;
    if (staged) {
      for (int32_t i = lane; i < len; i += 64) s_col[i] = a.col[b0 + i];
    }
    __builtin_amdgcn_s_waitcnt(0);  // the stores above are this wave's own: no barrier
    // 2) each output row: its segment in edge order
    int32_t b = b0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t t = ms + i;
      const uint32_t in = i + 1;
      const int32_t e = in < 64 ? __builtin_amdgcn_readlane(rp_lo, (int)in)
                                : (in < 128 ? __builtin_amdgcn_readlane(rp_hi, (int)(in - 64)) : a.rowptr[t + 1]);
      float acc = 0.f;
      int32_t k = b;
      if (staged) {
        for (; k + 8 <= e; k += 8) {  // indices in groups of 8 (LDS broadcast reads)
          int32_t q[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) q[j] = __builtin_amdgcn_readfirstlane(s_col[k - b0 + j]);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += from_src<SRC_CHUNKED>(a, xa, xb, q[j], ms, nr, c, cv);
        }
        for (; k < e; ++k)
          acc += from_src<SRC_CHUNKED>(a, xa, xb, __builtin_amdgcn_readfirstlane(s_col[k - b0]), ms, nr, c, cv);
      } else {
        for (; k < e; ++k)
          acc += from_src<SRC_CHUNKED>(a, xa, xb, __builtin_amdgcn_readfirstlane(a.col[k]), ms, nr, c, cv);
      }
      b = e;
      if (cv) {
        float v = acc;
        if (a.add0) v = a.add0[(int64_t)t * a.add0_ld + c] + v;
        if (a.add1) v = v + a.add1[(int64_t)t * a.add1_ld + c];
        a.out[(int64_t)t * a.out_ld + c] = v;
      }
    }
    ms = me;  // the next molecule starts where this one ends (R1 <= R0 + 64: no rescan needed)
  }
}

}  // namespace

// Opt-in (AIMX_HOP_REGS=1): bit-exact, but measured 4-12x SLOWER than hop_rows.hip in the step's
// own layout (c4 forward 123.7 vs 30.3 us, c5 519.5 vs 42.3 us; profiles/r05_hop_regs_ab.txt):
// every source is a dependent chain (LDS index read -> readfirstlane -> s_set_gpr_idx -> v_mov)
// of one wave per SIMD, with nothing to overlap it. Kept for the record and its tests.
bool gather_regs_on() {
  static const bool on = [] {
    const char* e = getenv("AIMX_HOP_REGS");
    return e && atoi(e) != 0;
  }();
  return on;
}

// Rows [0, split) (split = out_rpc, the first output chunk) here; the rest by hop_rows.hip's big
// tiles. Requires the molecule ids (row_seg).
int launch_gather_regs(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out, int64_t out_ld,
                       int64_t out_rpc, int64_t out_cs, const float* add0, int64_t add0_ld, const float* add1,
                       int64_t add1_ld, const int64_t* row_seg, int64_t row_seg_stride, hipStream_t stream,
                       int32_t skip_tail) {
  if (!row_seg || rows <= 0 || D <= 0) return AIMX_EARG;
  if (rows >= (int64_t)INT32_MAX - 128 || src_rpc >= INT32_MAX || out_rpc >= INT32_MAX) return AIMX_EARG;
  // the molecule's 64-row register block is addressed by 32-bit byte offsets
  if (64 * src_ld + D >= (int64_t)1 << 29) return AIMX_EARG;
  const int64_t split = (out_rpc > 0 && out_rpc < rows) ? out_rpc : rows;
  RegsArgs a;
  a.src = src;
  a.src_ld = src_ld;
  a.src_cs = src_cs;
  a.src_rpc = make_fastdiv(src_rpc > 0 ? (uint32_t)src_rpc : 0);
  a.rowptr = rowptr;
  a.col = col;
  a.D = (uint32_t)D;
  a.ncb = (uint32_t)cdiv(D, 64);
  a.split = (uint32_t)split;
  a.out = out;
  a.out_ld = out_ld;
  a.add0 = add0;
  a.add0_ld = add0_ld;
  a.add1 = add1;
  a.add1_ld = add1_ld;
  a.seg = row_seg;
  a.seg_stride = row_seg_stride;
  const int64_t blocks = cdiv(split, kGW) * a.ncb;
  if (blocks >= (int64_t)INT32_MAX) return AIMX_EARG;
  if (src_rpc > 0)
    hipLaunchKernelGGL(k_gather_regs<true>, dim3((unsigned)blocks), dim3(64), 0, stream, a);
  else
    hipLaunchKernelGGL(k_gather_regs<false>, dim3((unsigned)blocks), dim3(64), 0, stream, a);
  AIMX_CHECK_LAUNCH();
  if (rows > split)  // the hop chunks past the first: big tiles only
    return launch_gather_rows(src, src_ld, src_rpc, src_cs, D, rowptr, col, rows, out, out_ld, out_rpc, out_cs, add0,
                              add0_ld, add1, add1_ld, row_seg, row_seg_stride, stream, skip_tail, false);
  return AIMX_OK;
}

}  // namespace aimx
