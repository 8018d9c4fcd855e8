// The hop: segmented gather-sum over a stable CSR (HBM-bound integer-indexed row traffic).
//
// Reference: ShellConvolutionLayer.message_passing, src/models/layers.py:133-167
//   aggregated = scatter_add(x[src % N], target, dim_size = num_hops * N)
// Here each output row t is produced by ONE owner (no atomics): it walks its CSR segment
// (edges with target t, ascending edge id) and sums the source rows in that order starting from
// +0.0f, which reproduces CPU ATen scatter_add_ bit for bit. Lanes run along the feature dim with
// VEC-wide (16/8/4-byte) loads; a 64-lane wave covers 64*VEC consecutive floats of the flattened
// [rows, D] output, so the stores are coalesced. A workgroup owns a tile of consecutive rows: it
// stages the tile's rowptr and col slices in LDS, then (when the tile's sources span few rows, as
// they do in a molecular batch) the source rows themselves, and sums from LDS; the compulsory HBM
// traffic is x once, the CSR once and the output once (SURVEY.md §8d algorithmic bytes). Measured
// at roofline size (tools/hop_micro.py): 1.46 ms -> 1.11 ms per launch for staging the sources.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "aimx_common.h"
#include "hop_common.h"

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

// Row tiles: a workgroup owns `tile_rows` consecutive output rows. It stages their rowptr slice and
// (when it fits) their whole col slice in LDS with two coalesced loads, so the per-output-element
// dependency chain is LDS -> gathered source row -> store instead of rowptr -> col -> row in HBM.
// A tile whose rows hold no edges (the reference's hop chunks >= 1 are all-empty, layers.py:154)
// becomes a pure streaming store. Gathers are issued 8 at a time with clamped (always valid)
// indices and summed with selects, so the sum is the ordered edge-order sum bit for bit.
constexpr int kMaxTileRows = 64;   // nominal rows per tile
constexpr int kAlignWin = 64;      // a segment-aligned tile cut moves at most this many rows
constexpr int kMaxRows = kMaxTileRows + kAlignWin;  // rows of one (aligned) tile
constexpr int kGroup = 8;      // gathers in flight per thread
constexpr int kColCap = 512;             // default staged col entries per tile (2 KiB)
constexpr int kStageBytes = 17 * 1024 + 512;  // default LDS for the staged source span
constexpr int kBigMul = 16;            // small tiles per big tile (measured: 8 -> 16 with interleave, -1.2 %)

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

// Same sum with the tile's source rows staged in LDS. In a molecular batch the sources of a tile's
// targets are rows of the same few molecules, so the tile's col values span a short row range
// [lo, hi]; each of those rows is gathered ~deg times (once per edge that names it). Loading the
// span once with coalesced loads and summing from LDS turns ~10 vector-L1 gathers per source row
// into one global load plus ds_read_b128s (the L1 tag/fill rate, not HBM, bounds the unstaged
// gather phase: TCP pending-stall ~55 % of cycles at roofline size).
// cols[] holds BYTE offsets of the staged rows (precomputed once per tile) and cols[zslot] the
// offset of an all-zero staged row: slots past a row's segment read the zero row, and adding +0.0f
// leaves the sum bit-identical (the running sum starts at +0.0f, so it is never -0.0f), so the
// edge loop needs no data selects, only an index select per edge.
template <int VEC>
__device__ __forceinline__ void tile_body_staged(const float* s_x, const FastDiv& upr, const int32_t* s_ptr,
                                                 const int32_t* cols, int32_t zslot, int32_t base, uint32_t r0,
                                                 uint32_t nr, float* __restrict__ out, int64_t out_ld,
                                                 const FastDiv& out_rpc, int64_t out_cs,
                                                 const float* __restrict__ add0, int64_t add0_ld,
                                                 const float* __restrict__ add1, int64_t add1_ld) {
  using T = typename VecT<VEC>::T;
  constexpr int kU = 4;  // LDS reads in flight per thread (8, or two items in lockstep: slower)
  const uint32_t units = nr * upr.d;
  const char* xb = reinterpret_cast<const char*>(s_x);
  const char* cb = reinterpret_cast<const char*>(cols);
  const int32_t zb = zslot * 4;
  if (add0 || add1) {
    // the residual terms' loads go out before the LDS sum and are consumed after it: unconditional
    // (an absent term reads the output row, dropped below), so no branch joins them to a wait
    for (uint32_t t = threadIdx.x; t < units; t += blockDim.x) {
      const uint32_t rl = fdiv(t, upr);
      const uint32_t ub = (t - rl * upr.d) * VEC * 4;
      const uint32_t u = ub / 4;
      const uint32_t r = r0 + rl;
      float* orow = out + row_off(r, out_ld, out_rpc, out_cs);
      const T q0 = *reinterpret_cast<const T*>((add0 ? add0 + (int64_t)r * add0_ld : orow) + u);
      const T q1 = *reinterpret_cast<const T*>((add1 ? add1 + (int64_t)r * add1_ld : orow) + u);
      const int32_t bb = (s_ptr[rl] - base) * 4, eb = (s_ptr[rl + 1] - base) * 4;
      T acc = vzero<T>();
      for (int32_t kb = bb; kb < eb; kb += 4 * kU) {
        T v[kU];
#pragma unroll
        for (int j = 0; j < kU; ++j) {
          const int32_t off = *reinterpret_cast<const int32_t*>(cb + ((kb + 4 * j < eb) ? kb + 4 * j : zb));
          v[j] = *reinterpret_cast<const T*>(xb + off + ub);
        }
#pragma unroll
        for (int j = 0; j < kU; ++j) vadd(acc, v[j]);
      }
      T s0 = q0;  // add0 + sum, then + add1: the order below
      vadd(s0, acc);
      if (add0) acc = s0;
      T s1 = acc;
      vadd(s1, q1);
      if (add1) acc = s1;
      *reinterpret_cast<T*>(orow + u) = acc;
    }
    return;
  }
  for (uint32_t t = threadIdx.x; t < units; t += blockDim.x) {
    const uint32_t rl = fdiv(t, upr);
    const uint32_t ub = (t - rl * upr.d) * VEC * 4;
    const uint32_t r = r0 + rl;
    // col slots in bytes: (kb + 4j < eb) ? kb + 4j : zb
    const int32_t bb = (s_ptr[rl] - base) * 4, eb = (s_ptr[rl + 1] - base) * 4;
    T acc = vzero<T>();
    for (int32_t kb = bb; kb < eb; kb += 4 * kU) {
      T v[kU];
#pragma unroll
      for (int j = 0; j < kU; ++j) {
        const int32_t off = *reinterpret_cast<const int32_t*>(cb + ((kb + 4 * j < eb) ? kb + 4 * j : zb));
        v[j] = *reinterpret_cast<const T*>(xb + off + ub);
      }
#pragma unroll
      for (int j = 0; j < kU; ++j) vadd(acc, v[j]);
    }
    const uint32_t u = ub / 4;
    if (add0) {
      T s = *reinterpret_cast<const T*>(add0 + (int64_t)r * add0_ld + u);
      vadd(s, acc);
      acc = s;
    }
    if (add1) vadd(acc, *reinterpret_cast<const T*>(add1 + (int64_t)r * add1_ld + u));
    *reinterpret_cast<T*>(out + row_off(r, out_ld, out_rpc, out_cs) + u) = acc;
  }
}

struct HopArgs {
  const float* src;
  int64_t src_ld, src_cs;
  FastDiv src_rpc, upr;
  const int32_t* rowptr;
  const int32_t* col;
  uint32_t rows, tile_rows;
  uint32_t split_rows;  // rows [0, split) in workgroups of one tile; rows [split, rows) in big tiles
  uint32_t nsmall;      // workgroups of the small-tile range
  uint32_t big_rows;    // rows per big tile (a multiple of tile_rows)
  uint32_t col_cap;     // staged col entries per tile (dynamic LDS)
  uint32_t xcap_rows;   // staged source rows that fit the dynamic LDS (0: no staging)
  float* out;
  int64_t out_ld, out_cs;
  FastDiv out_rpc;
  const float* add0;
  int64_t add0_ld;
  const float* add1;
  int64_t add1_ld;
  const int64_t* seg;  // optional segment (molecule) id per row of [0, split_rows)
  int64_t seg_stride;
  int32_t flat_zero;    // rows past split are one contiguous [rows - split, D] region, no adds
  int32_t nt_store;     // nontemporal stores for that fill
  int32_t skip_tail;    // big tiles in the trailing EMPTY hop chunks are not written (segment_gather_sum)
  int32_t interleave;   // spread the big tiles among the small ones (block order)
  int32_t spec_stage;   // segment-aligned tiles in two round trips (process_tile_seg)
};

// All LDS is dynamic, carved at 16-byte multiples (MI355X guide: a static __shared__ ahead of the
// dynamic region shifts its base off 16-B alignment and every ds_read_b128 replays at ~64 cycles).
struct HopLds {
  int32_t* ptr;   // [kMaxRows + 1]
  int32_t* lohi;  // [3] (also the two aligned cuts of a segment-aligned tile; [2] a big tile's skip flag)
};
constexpr int kLdsHead = 136;  // ints ahead of the col slice: ptr (129) + lohi (2), padded to 16 B

// Rows [first, first + span) of src into s_x (row stride D floats), plus an all-zero row at index
// span. kStageB units per thread per batch: every load of a batch is issued (clamped indices, always
// valid addresses) before the first LDS store waits for one; a load behind the row guard would make
// the compiler wait for each load at the guard's join (one memory round trip per unit per thread).
#ifndef AIMX_HOP_STAGEB
#define AIMX_HOP_STAGEB 3
#endif
constexpr int kStageB = AIMX_HOP_STAGEB;
// An empty asm that reads a loaded value: the loads of a batch cannot be sunk past it to their LDS
// stores (the 64-VGPR budget otherwise makes the scheduler interleave load, wait, store per unit).
__device__ __forceinline__ void hold(const float& v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void hold(const float2& v) { asm volatile("" ::"v"(v.x), "v"(v.y)); }
__device__ __forceinline__ void hold(const float4& v) { asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w)); }
__device__ __forceinline__ void hold(const int32_t& v) { asm volatile("" ::"v"(v)); }
// (t_begin: units below it were staged by the caller; the zero row is always written here)
template <int VEC, bool SRC_CHUNKED>
__device__ __forceinline__ void stage_span(const HopArgs& a, float* s_x, uint32_t first, uint32_t span,
                                           uint32_t t_begin = 0) {
  using T = typename VecT<VEC>::T;
  const int32_t D = (int32_t)(a.upr.d * VEC);
  for (uint32_t t = threadIdx.x; t < a.upr.d; t += blockDim.x)
    *reinterpret_cast<T*>(s_x + span * D + t * VEC) = vzero<T>();
  const uint32_t units = span * a.upr.d;
  for (uint32_t t0 = t_begin; t0 < units; t0 += kStageB * blockDim.x) {
    T v[kStageB];
#pragma unroll
    for (int b = 0; b < kStageB; ++b) {
      const uint32_t t = min(t0 + threadIdx.x + (uint32_t)b * blockDim.x, units - 1);
      const uint32_t rl = fdiv(t, a.upr);
      v[b] = *reinterpret_cast<const T*>(a.src + src_off<SRC_CHUNKED>(first + rl, a.src_ld, a.src_rpc, a.src_cs) +
                                         (t - rl * a.upr.d) * VEC);
    }
#pragma unroll
    for (int b = 0; b < kStageB; ++b) hold(v[b]);
#pragma unroll
    for (int b = 0; b < kStageB; ++b) {
      const uint32_t t = t0 + threadIdx.x + (uint32_t)b * blockDim.x;
      if (t < units) {
        const uint32_t rl = fdiv(t, a.upr);
        *reinterpret_cast<T*>(s_x + rl * D + (t - rl * a.upr.d) * VEC) = v[b];
      }
    }
  }
}

// One tile of nr <= tile_rows rows at r0 (called by the whole workgroup; leaves LDS reusable).
template <int VEC, bool SRC_CHUNKED>
// s_col / s_x point into the dynamic LDS (col_cap entries, then the staged rows). They are passed
// down as arguments, never stored in memory: a pointer loaded back from LDS is a generic pointer
// and its reads become flat loads through the vector-memory pipe instead of ds_reads.
__device__ __forceinline__ void process_tile(const HopArgs& a, HopLds& L, int32_t* s_col, float* s_x, uint32_t r0,
                                             uint32_t nr) {
  if (threadIdx.x <= nr) L.ptr[threadIdx.x] = a.rowptr[r0 + threadIdx.x];
  if (threadIdx.x == 0) {
    L.lohi[0] = INT32_MAX;
    L.lohi[1] = INT32_MIN;
  }
  __syncthreads();
  const int32_t base = L.ptr[0];
  const int32_t ncols = L.ptr[nr] - base;
  if (ncols == 0) {  // no edges: a streaming store of zeros (+ the fused residual terms)
    tile_body<VEC, true, SRC_CHUNKED>(a.src, a.src_ld, a.src_rpc, a.src_cs, a.upr, L.ptr, s_col, base, r0, nr, a.out,
                                      a.out_ld, a.out_rpc, a.out_cs, a.add0, a.add0_ld, a.add1, a.add1_ld, false);
  } else if ((uint32_t)ncols > a.col_cap) {
    tile_body<VEC, false, SRC_CHUNKED>(a.src, a.src_ld, a.src_rpc, a.src_cs, a.upr, L.ptr, a.col, base, r0, nr, a.out,
                                       a.out_ld, a.out_rpc, a.out_cs, a.add0, a.add0_ld, a.add1, a.add1_ld, true);
  } else {
    int32_t lo = INT32_MAX, hi = INT32_MIN;
    for (int32_t i = threadIdx.x; i < ncols; i += blockDim.x) {
      const int32_t c = a.col[base + i];
      s_col[i] = c;
      lo = min(lo, c);
      hi = max(hi, c);
    }
    if (a.xcap_rows) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o, 64));
        hi = max(hi, __shfl_xor(hi, o, 64));
      }
      if ((threadIdx.x & 63) == 0) {
        atomicMin(&L.lohi[0], lo);
        atomicMax(&L.lohi[1], hi);
      }
    }
    __syncthreads();
    bool staged = false;
    if (a.xcap_rows) {
      lo = L.lohi[0];
      hi = L.lohi[1];
      // the span plus one zero row must fit, and one col slot is kept for the zero row's offset
      if ((uint32_t)(hi - lo) + 1 < a.xcap_rows && (uint32_t)ncols < a.col_cap) {
        staged = true;
        const int32_t D = (int32_t)(a.upr.d * VEC);
        const int32_t span = hi - lo + 1;
        // each thread rewrites the col entries it staged as byte offsets of the staged rows
        for (int32_t i = threadIdx.x; i < ncols; i += blockDim.x) s_col[i] = (s_col[i] - lo) * D * 4;
        if (threadIdx.x == 0) s_col[ncols] = span * D * 4;
        stage_span<VEC, SRC_CHUNKED>(a, s_x, (uint32_t)lo, (uint32_t)span);
        __syncthreads();
        tile_body_staged<VEC>(s_x, a.upr, L.ptr, s_col, ncols, base, r0, nr, a.out, a.out_ld, a.out_rpc, a.out_cs,
                              a.add0, a.add0_ld, a.add1, a.add1_ld);
      }
    }
    if (!staged)
      tile_body<VEC, true, SRC_CHUNKED>(a.src, a.src_ld, a.src_rpc, a.src_cs, a.upr, L.ptr, s_col, base, r0, nr, a.out,
                                        a.out_ld, a.out_rpc, a.out_cs, a.add0, a.add0_ld, a.add1, a.add1_ld, true);
  }
  __syncthreads();  // LDS is reused by the next tile of a big tile
}

// A segment-aligned tile (rows [0, split) with molecule ids) in two dependent global round trips
// instead of four: (1) the segment cuts together with the row pointers of every row the tile can
// span (the nominal range plus the 64-row cut window), (2) the tile's col slice together with a
// speculative stage of the tile's own source rows [r0, r0 + nr) -- in a molecular batch a
// molecule-aligned tile's sources are exactly its own rows. If the col range confirms it, the sum
// runs from that stage; otherwise the span is restaged as in process_tile (same result either way).
template <int VEC, bool SRC_CHUNKED>
__device__ __forceinline__ void process_tile_seg(const HopArgs& a, HopLds& L, int32_t* s_col, float* s_x,
                                                 uint32_t c0, uint32_t c1) {
  int32_t* spec = L.lohi + 2;  // [lo, hi] of the col slice (LDS head padding, see kLdsHead)
  {
    const uint32_t pend = min(c1 + (uint32_t)kAlignWin, a.split_rows);  // last possible cut
    for (uint32_t t = threadIdx.x; t <= pend - c0; t += blockDim.x) L.ptr[t] = a.rowptr[c0 + t];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w < 2) {
      const uint32_t c = w ? c1 : c0;
      uint32_t cut = c;
      if (c > 0 && c < a.split_rows) {
        const uint32_t q = min(c + lane, a.split_rows - 1);
        const int64_t sq = a.seg[(int64_t)q * a.seg_stride], sp = a.seg[(int64_t)(q - 1) * a.seg_stride];
        const unsigned long long m = __ballot((c + lane < a.split_rows) && sq != sp);
        if (m) cut = c + (uint32_t)__builtin_ctzll(m);
      }
      if (lane == 0) L.lohi[w] = (int32_t)cut;
    }
    if (threadIdx.x == 128) {
      spec[0] = INT32_MAX;
      spec[1] = INT32_MIN;
    }
  }
  __syncthreads();
  const uint32_t r0 = (uint32_t)L.lohi[0], r1 = (uint32_t)L.lohi[1];
  if (r1 <= r0) return;
  const uint32_t nr = r1 - r0;
  const int32_t* P = L.ptr + (r0 - c0);  // the tile's row pointers
  const int32_t base = P[0];
  const int32_t ncols = P[nr] - base;
  if (ncols == 0) {
    tile_body<VEC, true, SRC_CHUNKED>(a.src, a.src_ld, a.src_rpc, a.src_cs, a.upr, P, s_col, base, r0, nr, a.out,
                                      a.out_ld, a.out_rpc, a.out_cs, a.add0, a.add0_ld, a.add1, a.add1_ld, false);
    return;
  }
  if ((uint32_t)ncols >= a.col_cap || !a.xcap_rows || nr + 1 >= a.xcap_rows) {
    tile_body<VEC, false, SRC_CHUNKED>(a.src, a.src_ld, a.src_rpc, a.src_cs, a.upr, P, a.col, base, r0, nr, a.out,
                                       a.out_ld, a.out_rpc, a.out_cs, a.add0, a.add0_ld, a.add1, a.add1_ld, true);
    return;
  }
  const int32_t D = (int32_t)(a.upr.d * VEC);
  int32_t lo = INT32_MAX, hi = INT32_MIN;
  // the first kColB col entries and the first kStageB units of the speculative stage (rows [r0,
  // r0 + nr)) per thread go out together, unconditionally (clamped), held until all are issued: one
  // round trip for both; what is left (long col slices, tall tiles) follows in batches
#ifndef AIMX_HOP_COLB
#define AIMX_HOP_COLB 2
#endif
  constexpr int kColB = AIMX_HOP_COLB;
  {
    using T = typename VecT<VEC>::T;
    const uint32_t bd = blockDim.x, units = nr * a.upr.d;
    int32_t cv[kColB];
    T sv[kStageB];
#pragma unroll
    for (int b = 0; b < kColB; ++b) cv[b] = a.col[base + min((int32_t)(threadIdx.x + b * bd), ncols - 1)];
#pragma unroll
    for (int b = 0; b < kStageB; ++b) {
      const uint32_t t = min(threadIdx.x + (uint32_t)b * bd, units - 1);
      const uint32_t rl = fdiv(t, a.upr);
      sv[b] = *reinterpret_cast<const T*>(a.src + src_off<SRC_CHUNKED>(r0 + rl, a.src_ld, a.src_rpc, a.src_cs) +
                                          (t - rl * a.upr.d) * VEC);
    }
#pragma unroll
    for (int b = 0; b < kColB; ++b) hold(cv[b]);
#pragma unroll
    for (int b = 0; b < kStageB; ++b) hold(sv[b]);
#pragma unroll
    for (int b = 0; b < kColB; ++b) {
      const int32_t i = (int32_t)(threadIdx.x + b * bd);
      if (i < ncols) {
        s_col[i] = cv[b];
        lo = min(lo, cv[b]);
        hi = max(hi, cv[b]);
      }
    }
#pragma unroll
    for (int b = 0; b < kStageB; ++b) {
      const uint32_t t = threadIdx.x + (uint32_t)b * bd;
      if (t < units) {
        const uint32_t rl = fdiv(t, a.upr);
        *reinterpret_cast<T*>(s_x + rl * D + (t - rl * a.upr.d) * VEC) = sv[b];
      }
    }
  }
  for (int32_t i = threadIdx.x + kColB * blockDim.x; i < ncols; i += blockDim.x) {
    const int32_t c = a.col[base + i];
    s_col[i] = c;
    lo = min(lo, c);
    hi = max(hi, c);
  }
  stage_span<VEC, SRC_CHUNKED>(a, s_x, r0, nr, kStageB * blockDim.x);  // the rest and the zero row
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o, 64));
    hi = max(hi, __shfl_xor(hi, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&spec[0], lo);
    atomicMax(&spec[1], hi);
  }
  __syncthreads();
  lo = spec[0];
  hi = spec[1];
  uint32_t first = r0, span = nr;  // the staged rows
  bool staged = lo >= (int32_t)r0 && hi < (int32_t)(r0 + nr);
  if (!staged && (uint32_t)(hi - lo) + 1 < a.xcap_rows) {  // the guess missed: stage [lo, hi]
    __syncthreads();
    first = (uint32_t)lo;
    span = (uint32_t)(hi - lo + 1);
    stage_span<VEC, SRC_CHUNKED>(a, s_x, first, span);
    staged = true;
  }
  if (staged) {
    for (int32_t i = threadIdx.x; i < ncols; i += blockDim.x) s_col[i] = (s_col[i] - (int32_t)first) * D * 4;
    if (threadIdx.x == 0) s_col[ncols] = (int32_t)span * D * 4;
    __syncthreads();
    tile_body_staged<VEC>(s_x, a.upr, P, s_col, ncols, base, r0, nr, a.out, a.out_ld, a.out_rpc, a.out_cs, a.add0,
                          a.add0_ld, a.add1, a.add1_ld);
  } else {
    tile_body<VEC, true, SRC_CHUNKED>(a.src, a.src_ld, a.src_rpc, a.src_cs, a.upr, P, s_col, base, r0, nr, a.out,
                                      a.out_ld, a.out_rpc, a.out_cs, a.add0, a.add0_ld, a.add1, a.add1_ld, true);
  }
}

// Rows [0, split) (the first output chunk) run one tile per workgroup: separate workgroups overlap
// their load phases better than tiles walked in sequence. Rows [split, rows) (hop chunks >= 1)
// run in big tiles: a big tile whose rows hold no edges at all (the reference's chunks >= 1 are
// empty, layers.py:154) is one long streaming store, so the two thirds of the output that are zero
// cost stores, not workgroup launches; a big tile with edges walks its tiles in order.
template <int VEC, bool SRC_CHUNKED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_gather_sum(const HopArgs a) {
  // [ptr | lohi | pad] [col_cap col entries] [xcap_rows x D staged rows]
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  HopLds L{s_dyn, s_dyn + kMaxRows + 1};
  int32_t* s_col = s_dyn + kLdsHead;
  float* s_x = reinterpret_cast<float*>(s_dyn + kLdsHead + a.col_cap);
  // Block order: with `interleave`, the big (mostly zero-fill) tiles are spread evenly among the
  // gather tiles, so the chip runs the write-bound fill beside the latency-bound gathers instead
  // of one phase after the other. big(b) = # big blocks among 0..b = floor((b+1) nbig / total).
  uint32_t bsmall = blockIdx.x, bbig = 0;
  bool is_small = blockIdx.x < a.nsmall;
  if (a.interleave) {
    const uint64_t total = (uint64_t)gridDim.x, nbig = total - a.nsmall;
    const uint32_t c1 = (uint32_t)(((uint64_t)blockIdx.x + 1) * nbig / total);
    const uint32_t c0 = (uint32_t)((uint64_t)blockIdx.x * nbig / total);
    is_small = (c1 == c0);
    bsmall = blockIdx.x - c1;
    bbig = c1 - 1;
  } else if (!is_small) {
    bbig = blockIdx.x - a.nsmall;
  }
  if (is_small) {
    uint32_t r0 = bsmall * a.tile_rows;
    uint32_t r1 = min(r0 + a.tile_rows, a.split_rows);
    if (a.seg && a.spec_stage) {
      process_tile_seg<VEC, SRC_CHUNKED>(a, L, s_col, s_x, r0, r1);
      return;
    }
    if (a.seg) {
      // Segment-aligned cuts: each nominal cut c moves to the first segment (molecule) start in
      // [c, c + 64) (c itself if none), so a tile holds whole molecules and its source rows are
      // exactly its own rows: x is staged once instead of once per straddling tile. Both cuts
      // are the same function of c, so consecutive tiles still partition the rows exactly.
      const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
      if (w < 2) {
        const uint32_t c = w ? r1 : r0;
        uint32_t cut = c;
        if (c > 0 && c < a.split_rows) {
          const uint32_t q = min(c + lane, a.split_rows - 1);
          const int64_t sq = a.seg[(int64_t)q * a.seg_stride], sp = a.seg[(int64_t)(q - 1) * a.seg_stride];
          const unsigned long long m = __ballot((c + lane < a.split_rows) && sq != sp);
          if (m) cut = c + (uint32_t)__builtin_ctzll(m);
        }
        if (lane == 0) L.lohi[w] = (int32_t)cut;
      }
      __syncthreads();
      r0 = (uint32_t)L.lohi[0];
      r1 = (uint32_t)L.lohi[1];
      __syncthreads();
    }
    if (r1 > r0) process_tile<VEC, SRC_CHUNKED>(a, L, s_col, s_x, r0, r1 - r0);
    return;
  }
  const uint32_t R0 = a.split_rows + bbig * a.big_rows;
  const uint32_t NR = min(a.big_rows, a.rows - R0);
  if (threadIdx.x == 0) {
    L.lohi[0] = a.rowptr[R0];
    L.lohi[1] = a.rowptr[R0 + NR];
    // skip_tail: no edge from the start of R0's chunk to the end (every consumer trims those chunks)
    L.lohi[2] = a.skip_tail && a.out_rpc.d > 0 && a.rowptr[fdiv(R0, a.out_rpc) * a.out_rpc.d] == a.rowptr[a.rows];
  }
  __syncthreads();
  if (L.lohi[2]) return;
  if (L.lohi[0] == L.lohi[1]) {
    if (a.flat_zero) {
      // the big tile's rows are one contiguous [NR, D] region and there is nothing to add: a flat
      // streaming fill (16-byte stores, no per-element row arithmetic; nontemporal when asked)
      typedef float V __attribute__((ext_vector_type(VEC)));
      V* o = reinterpret_cast<V*>(a.out + (int64_t)R0 * a.out_ld);
      const uint32_t n = NR * a.upr.d;
      const V z = (V)(0.f);
      if (a.nt_store) {
        for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) __builtin_nontemporal_store(z, o + t);
      } else {
        for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) o[t] = z;
      }
      return;
    }
    tile_body<VEC, true, SRC_CHUNKED>(a.src, a.src_ld, a.src_rpc, a.src_cs, a.upr, L.ptr, s_col, 0, R0, NR, a.out,
                                      a.out_ld, a.out_rpc, a.out_cs, a.add0, a.add0_ld, a.add1, a.add1_ld, false);
    return;
  }
  __syncthreads();
  for (uint32_t r0 = R0; r0 < R0 + NR; r0 += a.tile_rows)
    process_tile<VEC, SRC_CHUNKED>(a, L, s_col, s_x, r0, min(a.tile_rows, R0 + NR - r0));
}

inline bool aligned(const void* p, int bytes) { return ((uintptr_t)p % bytes) == 0; }

// The launcher's tuning knobs (opt_i64: defaults in the product library; -1 = the launcher's own
// default), read once per process (an eager step calls the launcher ~6 times)
struct HopEnv {
  int64_t tile_units, big_mul, col_cap, stage_bytes, flat, nt, interleave, spec;
  bool no_seg;
};
const HopEnv& hop_env() {
  static const HopEnv e = [] {
    HopEnv v;
    v.tile_units = tune_i64("AIMX_HOP_TILE_UNITS", -1);
    v.big_mul = tune_i64("AIMX_HOP_BIG_MUL", -1);
    v.col_cap = tune_i64("AIMX_HOP_COL_CAP", -1);
    v.stage_bytes = tune_i64("AIMX_HOP_STAGE_BYTES", -1);
    v.flat = tune_i64("AIMX_HOP_FLAT", 1);
    v.nt = tune_i64("AIMX_HOP_NT", 0);
    v.interleave = tune_i64("AIMX_HOP_INTERLEAVE", 1);
    v.spec = tune_i64("AIMX_HOP_SPEC", 1);
    v.no_seg = tune_i64("AIMX_HOP_NO_SEG", 0) != 0;
    return v;
  }();
  return e;
}

}  // namespace
}  // namespace aimx

using namespace aimx;

namespace aimx {
// aimx_segment_gather_sum with skip_tail: the big tiles of output chunks that lie wholly in the
// trailing run of edge-less chunks are not written (the message-passing stack: its GEMMs trim those
// columns of F exactly, AimxGemmArgs.zc_*, so the zeros the reference's hop leaves there are never
// read)
int segment_gather_sum(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out, int64_t out_ld,
                       int64_t out_rpc, int64_t out_cs, const float* add0, int64_t add0_ld, const float* add1,
                       int64_t add1_ld, const int64_t* row_seg, int64_t row_seg_stride, hipStream_t stream,
                       int32_t skip_tail) {
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
  // Launch size: the kernels index threads and rows in 32 bits. A call past that (a very large
  // inference batch) runs as consecutive row ranges, each inside one output chunk: a range's row
  // pointers, output rows, residual rows and molecule ids are offsets of the caller's (rows are
  // independent sums, so the result is the one-launch result, bit for bit).
  // (the odd-width kernel indexes threads within a tile and rows in 32 bits: only rows < 2^31 bound
  // it; the aligned kernel's flat thread index also spans rows x D / vec. A split call loses the
  // chunked fast paths — zero-fill tiles, skip_tail — so the cap must not bite at configured sizes:
  // c5's 6-hop forward at roofline size is 6.6 M rows of 307.)
  {
    const int64_t upr_v = vec < 4 ? 1 : cdiv(D, vec);
    int64_t cap = std::max<int64_t>(1, ((int64_t)INT32_MAX - 1) / std::max<int64_t>(upr_v, 1) / 2);
    if (const int64_t f = opt_i64("AIMX_HOP_MAX_ROWS", 0)) cap = std::min(cap, f);  // test hook
    const int64_t rpc = (out_rpc > 0 && out_rpc < rows) ? out_rpc : rows;
    if (rows > cap) {
      for (int64_t r0 = 0; r0 < rows;) {
        const int64_t in_chunk = rpc - r0 % rpc;              // rows left in r0's output chunk
        const int64_t n = std::min<int64_t>({cap, in_chunk, rows - r0});
        float* o = out + (r0 % rpc) * out_ld + (r0 / rpc) * (rpc < rows ? out_cs : 0);
        const bool first = r0 < rpc;                             // row_seg covers the first chunk
        const int rc = segment_gather_sum(src, src_ld, src_rpc, src_cs, D, rowptr + r0, col, n, o, out_ld, 0, 0,
                                          add0 ? add0 + r0 * add0_ld : nullptr, add0_ld,
                                          add1 ? add1 + r0 * add1_ld : nullptr, add1_ld,
                                          first && row_seg ? row_seg + r0 * row_seg_stride : nullptr, row_seg_stride,
                                          stream, 0);
        if (rc != AIMX_OK) return rc;
        r0 += n;
      }
      return AIMX_OK;
    }
  }
  // rows that are not runs of 16-byte-aligned vectors (odd D, unaligned chunk offsets) take the
  // 16-byte-at-4-byte-alignment kernel (hop_unal.hip)
  const HopEnv& E = hop_env();
  if (vec < 4)
    return launch_gather_unal(src, src_ld, src_rpc, src_cs, D, rowptr, col, rows, out, out_ld, out_rpc, out_cs,
                              add0, add0_ld, add1, add1_ld, row_seg, row_seg_stride, stream, skip_tail);
  const int64_t upr_i = D / vec;
  // 32-bit thread indexing (rows * D / vec < 2^31) and int32 chunked row ids.
  if (rows * upr_i >= (int64_t)INT32_MAX || src_rpc >= INT32_MAX || out_rpc >= INT32_MAX) return AIMX_EARG;
  const int threads = 256;
  // tile height: ~2 vector units per thread, then shorter tiles while the grid is under 4
  // workgroups per CU (small batches are latency-bound: more workgroups hide more latency)
  // (rows of 129..256 vector units, c4's D = 153: two units per thread left 3-row tiles; 4 per
  // thread measured 20 us faster per c4 step, neutral at c2 and slower at c5's 307-wide rows —
  // profiles/r02_hop_tile_ab.txt; results never depend on the tiling)
  const int64_t tile_units = E.tile_units >= 0 ? E.tile_units : ((upr_i > 128 && upr_i <= 256) ? 4 * threads : 2 * threads);
  int64_t tr = std::min<int64_t>(kMaxTileRows, std::max<int64_t>(1, tile_units / upr_i));
  while (tr > 1 && cdiv(rows, tr) < 1024) tr = std::max<int64_t>(1, tr / 2);
  // output rows past the first chunk (hop chunks >= 1; out_rpc = rows per chunk) go in big tiles
  // once those rows hold >= 2048 tiles (8 per CU) to spare
  const int64_t split = (out_rpc > 0 && out_rpc < rows) ? out_rpc : rows;
  const int64_t big_max = std::max<int64_t>(1, (E.big_mul >= 0 ? E.big_mul : kBigMul));
  const int64_t big_mul = std::max<int64_t>(1, std::min<int64_t>(big_max, cdiv(rows - split, tr) / 2048));
  const int64_t big = tr * big_mul;
  const int64_t nsmall = cdiv(split, tr);
  const int64_t blocks = nsmall + cdiv(rows - split, big);
  // LDS budget for the staged source span (AIMX_HOP_STAGE_BYTES overrides; 0 disables staging)
  // (the defaults keep 8 workgroups = 32 waves per CU resident: <= 20 KiB of LDS each)
  const int64_t col_cap = (std::max<int64_t>(64, (E.col_cap >= 0 ? E.col_cap : kColCap)) + 3) / 4 * 4;
  const int64_t stage_bytes = (E.stage_bytes >= 0 ? E.stage_bytes : kStageBytes);
  int64_t xcap = stage_bytes / (4 * D);
  if (xcap < 2) xcap = 0;
  xcap = std::min<int64_t>(xcap, 4096);
  const size_t dyn = (size_t)((kLdsHead + col_cap) * 4 + xcap * D * 4);
  HopArgs a;
  a.src = src;
  a.src_ld = src_ld;
  a.src_cs = src_cs;
  a.src_rpc = make_fastdiv(src_rpc > 0 ? (uint32_t)src_rpc : 0);
  a.upr = make_fastdiv((uint32_t)upr_i);
  a.rowptr = rowptr;
  a.col = col;
  a.rows = (uint32_t)rows;
  a.tile_rows = (uint32_t)tr;
  a.split_rows = (uint32_t)split;
  a.nsmall = (uint32_t)nsmall;
  a.big_rows = (uint32_t)big;
  a.col_cap = (uint32_t)col_cap;
  a.xcap_rows = (uint32_t)xcap;
  a.out = out;
  a.out_ld = out_ld;
  a.out_cs = out_cs;
  a.out_rpc = make_fastdiv(out_rpc > 0 ? (uint32_t)out_rpc : 0);
  a.add0 = add0;
  a.add0_ld = add0_ld;
  a.add1 = add1;
  a.add1_ld = add1_ld;
  // segment-aligned tiles: only for the one-tile-per-workgroup range, and only when the staged
  // source span is in use (the alignment is what makes the span equal the tile)
  // (tiles of >= 16 rows only: moving a cut of a 3-row tile up to a 40-atom molecule start turns
  // most tiles empty and the rest too tall to stage — c4/c5 measured 6-20 % slower)
  a.seg = (row_seg && xcap > 0 && tr >= 16 && !E.no_seg) ? row_seg : nullptr;
  a.seg_stride = row_seg_stride;
  // chunks >= 1 contiguous after chunk 0 (a plain [h*N, D] output, as the hop op writes it)
  const bool contiguous = out_ld == D && (out_rpc <= 0 || out_cs == out_rpc * out_ld);
  a.flat_zero = (contiguous && !add0 && !add1 && E.flat != 0) ? 1 : 0;
  a.nt_store = E.nt != 0 ? 1 : 0;
  a.interleave = E.interleave != 0 ? 1 : 0;
  a.spec_stage = E.spec != 0 ? 1 : 0;
  a.skip_tail = skip_tail;
  using KFn = void (*)(const HopArgs);
  const bool chunked = src_rpc > 0;
  KFn fn = vec == 4 ? (chunked ? k_gather_sum<4, true> : k_gather_sum<4, false>)
           : vec == 2 ? (chunked ? k_gather_sum<2, true> : k_gather_sum<2, false>)
                      : (chunked ? k_gather_sum<1, true> : k_gather_sum<1, false>);
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(threads), dyn, stream, a);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
}  // namespace aimx

extern "C" int aimx_segment_gather_sum(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out,
                                       int64_t out_ld, int64_t out_rpc, int64_t out_cs, const float* add0,
                                       int64_t add0_ld, const float* add1, int64_t add1_ld, const int64_t* row_seg,
                                       int64_t row_seg_stride, aimx_stream_t stream) {
  return aimx::segment_gather_sum(src, src_ld, src_rpc, src_cs, D, rowptr, col, rows, out, out_ld, out_rpc, out_cs,
                                  add0, add0_ld, add1, add1_ld, row_seg, row_seg_stride, (hipStream_t)stream, 0);
}

extern "C" int aimx_segment_gather_sum_ex(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs,
                                          int64_t D, const int32_t* rowptr, const int32_t* col, int64_t rows,
                                          float* out, int64_t out_ld, int64_t out_rpc, int64_t out_cs,
                                          const float* add0, int64_t add0_ld, const float* add1, int64_t add1_ld,
                                          const int64_t* row_seg, int64_t row_seg_stride, int32_t flags,
                                          aimx_stream_t stream) {
  if (flags & ~AIMX_GATHER_SKIP_TAIL) return AIMX_EARG;
  return aimx::segment_gather_sum(src, src_ld, src_rpc, src_cs, D, rowptr, col, rows, out, out_ld, out_rpc, out_cs,
                                  add0, add0_ld, add1, add1_ld, row_seg, row_seg_stride, (hipStream_t)stream,
                                  (flags & AIMX_GATHER_SKIP_TAIL) ? 1 : 0);
}
