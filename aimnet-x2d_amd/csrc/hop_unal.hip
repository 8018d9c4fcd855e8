// The hop for rows that are not runs of 16-byte-ALIGNED vectors (odd widths D = int(0.3 * hidden):
// 153 / 307 at hidden 512 / 1024, reference src/models/gnn.py:100; hop chunks at column offset D of
// the concatenated [x | chunk_0 | ...] matrix, layers.py:76-79), by 16-byte vectors at 4-byte-aligned
// addresses. Same contract and bit-exact result as hop.hip (the ordered edge-order sum
// of CPU scatter_add_, layers.py:133-167).
//
// gfx950 executes global_load/store_dwordx4 at any 4-byte-aligned address (LLVM emits them for a
// 4-byte-aligned 16-byte struct on this target; tools/micro/unal_copy.hip checks the copy bit for bit
// and its rate). A row is then read and written as units of 4 columns [4g, 4g + 4) from the row's
// own start, whatever its alignment: the 16 bytes at min(c, D - 4) are always inside the row, and
// the last, partial unit's lanes are moved into place (staging: written shifted into LDS; residual
// terms: selects); its stores take dwords. In LDS the staged units sit 16-byte aligned, so the sum
// is ds_read_b128 throughout, and there is no realignment tile (round 3's hop_rows.hip, removed in round
// 6: stage -> sum -> shift through LDS -> store, four barriers per 80-column pass in sequence).
//
// Work split, as hop.hip's: a workgroup owns a segment-aligned tile (the molecules that start in its
// nominal window; sources are then the tile's own rows, staged speculatively) and ONE column slice
// of it. The slices of one tile are separate workgroups on one XCD (same L2 for the shared row
// pointers and col slice, the only bytes read twice), so a wide row costs parallel workgroups, not
// sequential passes. Round trips per workgroup: row pointers + molecule cuts, the col slice, the
// stage; each a batch of unconditional loads held in registers until all are out (a guarded load
// per entry made hipcc wait for each one). The backward's residual terms are loaded before the LDS
// sum. Hop chunks >= 1 (no edges for reference inputs) are big streaming tiles among the windows.
// Measured variants and why the defaults: DESIGN.md §3 "the odd-width hop", profiles/r05_hop_unal_ab.txt.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "aimx_common.h"
#include "hop_common.h"

namespace aimx {
namespace {

constexpr int kUT = 256;          // threads per workgroup
constexpr int kUMaxTile = 64;     // nominal rows per tile (upper bound)
constexpr int kUAlignWin = 64;    // a segment-aligned cut moves at most this many rows
constexpr int kUMaxRows = kUMaxTile + kUAlignWin;
constexpr int kUHead = 136;       // ints ahead of the col slice: row pointers [129] + misc [4], 16-byte multiple
constexpr int kUMisc = 129;       // misc words: [0] lo / cut0, [1] hi / cut1, [2] spec lo, [3] spec hi
constexpr int kUGroup = 4;        // LDS reads in flight per thread

// Workgroup barrier for LDS hand-offs: waits for this wave's LDS operations only. __syncthreads()'s
// fence also waits vmcnt(0), draining every global load in flight (loads in flight);
// no thread here reads another thread's global writes, and an LDS store of loaded data already
// waits for that load.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct __attribute__((packed, aligned(4))) F4u {
  float x, y, z, w;
};

__device__ __forceinline__ float4 f4z() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void f4acc(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}

// Columns [c, c + 4) of a row of width D (c < D): one 16-byte load at the row's 4-byte alignment,
// or dwords for the row's last, partial unit (never past the row's end).
__device__ __forceinline__ float4 ld_unit(const float* row, uint32_t c, uint32_t D) {
  if (c + 4 <= D) {
    const F4u v = *reinterpret_cast<const F4u*>(row + c);
    return make_float4(v.x, v.y, v.z, v.w);
  }
  float4 v = f4z();
  v.x = row[c];
  if (c + 1 < D) v.y = row[c + 1];
  if (c + 2 < D) v.z = row[c + 2];
  return v;
}
// The 16 bytes of a row at columns [min(c, D - 4), +4) (D >= 4: always inside the row), as one load:
// all four lanes are consumed unconditionally (put_unit), so the compiler neither splits nor
// predicates it, and a batch of them stays in flight together.
__device__ __forceinline__ float4 ld_raw(const float* row, uint32_t c, uint32_t D) {
  const F4u v = *reinterpret_cast<const F4u*>(row + min(c, D - 4));
  return make_float4(v.x, v.y, v.z, v.w);
}
// ld_raw's 16 bytes as columns c.. of the row: lanes moved down by sh = c - min(c, D - 4) (0 for a
// full unit; the lanes past the row's end then hold other columns, never stored)
// (two-level selects on the shift's bits: a select chain on sh == 0 / 1 / 2 becomes a private-memory
// table indexed by sh)
__device__ __forceinline__ float4 shift_down(const float4 v, uint32_t sh) {
  const bool b1 = (sh & 1u) != 0, b2 = (sh & 2u) != 0;
  const float x = v.x, y = v.y, z = v.z, w = v.w;  // scalars: a select of member addresses keeps v in memory
  float4 r;
  r.x = b2 ? (b1 ? w : z) : (b1 ? y : x);
  r.y = b2 ? w : (b1 ? z : y);
  r.z = (b1 || b2) ? w : z;
  r.w = w;
  return r;
}
// ld_raw's 16 bytes into a staged row d (slice column 0 at d[0]) at slice column min(c, D - 4) - 4 u0:
// a full unit lands on its own 16 bytes; the last, partial unit of an odd-width row lands shifted
// down, rewriting the same values over columns of the unit before it (identical bytes).
__device__ __forceinline__ void put_raw(float* d, uint32_t c, uint32_t D, uint32_t u0, const float4& v) {
  float* q = d + (min(c, D - 4) - 4 * u0);
  q[0] = v.x;
  q[1] = v.y;
  q[2] = v.z;
  q[3] = v.w;
}
__device__ __forceinline__ void st_unit(float* row, uint32_t c, uint32_t D, const float4& v) {
  if (c + 4 <= D) {
    *reinterpret_cast<F4u*>(row + c) = F4u{v.x, v.y, v.z, v.w};
    return;
  }
  row[c] = v.x;
  if (c + 1 < D) row[c + 1] = v.y;
  if (c + 2 < D) row[c + 2] = v.z;
}

struct UnalArgs {
  const float* src;
  int64_t src_ld, src_cs;
  FastDiv src_rpc;
  const int32_t* rowptr;
  const int32_t* col;
  uint32_t D, upr;            // row width; units (4 columns) per row
  uint32_t slices, cu;        // column slices per tile; units per slice (the last may be shorter)
  uint32_t pitch, pitch_l2;   // staged row stride in units (a power of two, >= cu, a multiple of 16)
  int32_t compact;            // thread t owns unit t % cs.d of row t / cs.d instead (row stride cu units)
  FastDiv cu_full, cu_last;   // units of a full / the last slice
  FastDiv upr_f;              // units of a whole row (big tiles)
  uint32_t rows, split;       // tiles cover rows [0, split); big tiles rows [split, rows)
  uint32_t tile_rows, ntiles, nsmall;
  uint32_t big_rows, nbig;
  uint32_t col_cap, xcap;     // staged col entries; staged rows (incl. the zero row) per workgroup
  int32_t interleave, flat_zero, skip_tail;
  float* out;
  int64_t out_ld, out_cs;
  FastDiv out_rpc;
  const float* add0;
  int64_t add0_ld;
  const float* add1;
  int64_t add1_ld;
  const int64_t* seg;  // molecule id per row of [0, split) (optional)
  int64_t seg_stride;
  // the residual rows for the prefetching sum (ADDS): add0 / add1, or src row 0 (never used) when absent
  const float* q0;
  int64_t q0_ld;
  const float* q1;
  int64_t q1_ld;
};

// make_fastdiv on the device (d < 2^31)
__device__ __forceinline__ FastDiv fastdiv_dev(uint32_t d) {
  FastDiv f{d, 0, 0};
  if (d == 0) return f;
  while ((1u << f.l) < d) ++f.l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << f.l) - d)) / d) + 1);
  return f;
}

template <bool SRC_CHUNKED>
__device__ __forceinline__ const float* src_row(const UnalArgs& a, uint32_t q) {
  if (!SRC_CHUNKED) return a.src + (int64_t)q * a.src_ld;
  const uint32_t k = fdiv(q, a.src_rpc);
  return a.src + (int64_t)(q - k * a.src_rpc.d) * a.src_ld + (int64_t)k * a.src_cs;
}

// The residual terms and the store of unit (row r, columns c..c+3): out = add0 + sum + add1 (the
// order hop.hip uses).
__device__ __forceinline__ void finish_unit(const UnalArgs& a, uint32_t r, uint32_t c, float4 acc) {
  if (a.add0) {
    float4 s = ld_unit(a.add0 + (int64_t)r * a.add0_ld, c, a.D);
    f4acc(s, acc);
    acc = s;
  }
  if (a.add1) f4acc(acc, ld_unit(a.add1 + (int64_t)r * a.add1_ld, c, a.D));
  st_unit(a.out + row_off(r, a.out_ld, a.out_rpc, a.out_cs), c, a.D, acc);
}

// Rows [r0, r0 + nr), units [u0, u0 + cs.d) of the slice, summed straight from global memory (tiles
// whose col slice or source span does not fit LDS, and edge-less tiles: cols == nullptr).
template <bool SRC_CHUNKED>
__device__ __forceinline__ void rows_global(const UnalArgs& a, const int32_t* P, const int32_t* cols, int32_t base,
                                            uint32_t r0, uint32_t nr, uint32_t u0, const FastDiv& cs) {
  const uint32_t units = nr * cs.d;
  for (uint32_t t = threadIdx.x; t < units; t += kUT) {
    const uint32_t rl = fdiv(t, cs);
    const uint32_t c = 4 * (u0 + t - rl * cs.d);
    float4 acc = f4z();
    if (cols) {
      const int32_t b = P[rl] - base, e = P[rl + 1] - base;
      for (int32_t k = b; k < e; ++k) f4acc(acc, ld_unit(src_row<SRC_CHUNKED>(a, (uint32_t)cols[k]), c, a.D));
    }
    finish_unit(a, r0 + rl, c, acc);
  }
}

// Rows [first, first + span), units [u0, u0 + cs.d) into s_x (row stride wsu units, 16-byte aligned),
// plus an all-zero row at index span. dwords: ld_unit for every unit (a sub-slice may start at the
// partial last unit, which put_raw would write in front of the row). kSB units per thread per batch: every load of a batch is issued
// (clamped, always valid addresses) before the first LDS store waits for one. (D >= 4 takes ld_raw /
// put_raw: the launcher keeps a partial last unit out of a slice of its own.)
#ifndef AIMX_HOPU_SB
#define AIMX_HOPU_SB 4
#endif
#ifndef AIMX_HOPU_CB
#define AIMX_HOPU_CB 4
#endif
#ifndef AIMX_HOPU_COMB
#define AIMX_HOPU_COMB 0
#endif
constexpr int kSB = AIMX_HOPU_SB;
constexpr int kCB = AIMX_HOPU_CB;  // col entries per thread per batch (tile)
// An empty asm that reads a loaded value: a batch's loads cannot be sunk past it to their uses, so
// they stay in flight together instead of one wait per load.
__device__ __forceinline__ void hold(const int32_t& v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void hold(const float4& v) { asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w)); }
template <bool SRC_CHUNKED>
__device__ __forceinline__ void stage(const UnalArgs& a, float* s_x, uint32_t first, uint32_t span, uint32_t u0,
                                      const FastDiv& cs, uint32_t wsu, bool dwords) {
  const uint32_t ws = 4 * wsu;
  for (uint32_t t = threadIdx.x; t < wsu; t += kUT) reinterpret_cast<float4*>(s_x + span * ws)[t] = f4z();
  const uint32_t units = span * cs.d;
  if (a.D < 4 || dwords) {
    for (uint32_t t = threadIdx.x; t < units; t += kUT) {
      const uint32_t rl = fdiv(t, cs);
      const uint32_t k = t - rl * cs.d;
      *reinterpret_cast<float4*>(s_x + rl * ws + 4 * k) = ld_unit(src_row<SRC_CHUNKED>(a, first + rl), 4 * (u0 + k), a.D);
    }
    return;
  }
  for (uint32_t t0 = 0; t0 < units; t0 += kSB * kUT) {
    float4 v[kSB];
#pragma unroll
    for (int b = 0; b < kSB; ++b) {
      const uint32_t t = min(t0 + threadIdx.x + (uint32_t)b * kUT, units - 1);
      const uint32_t rl = fdiv(t, cs);
      v[b] = ld_raw(src_row<SRC_CHUNKED>(a, first + rl), 4 * (u0 + t - rl * cs.d), a.D);
    }
#pragma unroll
    for (int b = 0; b < kSB; ++b) hold(v[b]);
#pragma unroll
    for (int b = 0; b < kSB; ++b) {
      const uint32_t t = t0 + threadIdx.x + (uint32_t)b * kUT;
      if (t < units) {
        const uint32_t rl = fdiv(t, cs);
        put_raw(s_x + rl * ws, 4 * (u0 + t - rl * cs.d), a.D, u0, v[b]);
      }
    }
  }
}

// Rows [r0, r0 + nr) of the slice, summed from the staged rows: P[0..nr] their row pointers, col
// entries from P[0] = pbase on as byte offsets into xb (cb), an all-zero staged row at byte offset
// *(cb + zb). Thread t owns unit t % pitch of row t / pitch (lanes past the slice's units idle):
// with a 16-unit multiple pitch and a 256-byte multiple row stride every unit k sits in 16-byte slot
// k % 16 = lane % 16 of the LDS banks, whatever row its source is, so each ds_read_b128 lane group
// ({0-3,12-15,20-27}, ...: distinct lane % 16) reads distinct slots: no bank conflict.
// The residual terms and the store of unit c of row r from a prefetched pair of raw loads (ADDS).
__device__ __forceinline__ void finish_pre(const UnalArgs& a, uint32_t r, uint32_t c, const float4& q0,
                                           const float4& q1, float4 acc) {
  const uint32_t sh = c - min(c, a.D - 4);  // the partial last unit's shift (0 otherwise)
  float4 s0 = shift_down(q0, sh);
  f4acc(s0, acc);
  if (a.add0) acc = s0;
  float4 s1 = acc;
  f4acc(s1, shift_down(q1, sh));
  if (a.add1) acc = s1;
  st_unit(a.out + row_off(r, a.out_ld, a.out_rpc, a.out_cs), c, a.D, acc);
}

template <bool ADDS>
__device__ __forceinline__ void sum_rows(const UnalArgs& a, const int32_t* P, int32_t pbase, const char* cb,
                                         const char* xb, int32_t zb, uint32_t r0, uint32_t nr, uint32_t u0,
                                         const FastDiv& cs, bool compact) {
  const uint32_t units = compact ? nr * cs.d : nr << a.pitch_l2;
  constexpr bool pre = ADDS;  // residual terms prefetched (the launcher: D >= 4 and a term present)
  for (uint32_t t = threadIdx.x; t < units; t += kUT) {
    const uint32_t rl = compact ? fdiv(t, cs) : t >> a.pitch_l2;
    const uint32_t k = compact ? t - rl * cs.d : t & (a.pitch - 1);
    if (k >= cs.d) continue;
    const uint32_t c = 4 * (u0 + k);
    const uint32_t r = r0 + rl;
    // the residual rows' 16 bytes go out before the LDS sum and are consumed after it: unconditional
    // loads (a missing term reads src row 0 instead, set up by the launcher, and is dropped), so no
    // branch joins them to a wait
    float4 q0, q1;
    if (pre) {
      q0 = ld_raw(a.q0 + (int64_t)r * a.q0_ld, c, a.D);
      q1 = ld_raw(a.q1 + (int64_t)r * a.q1_ld, c, a.D);
    }
    const uint32_t ub = 16 * k;
    const int32_t bb = (P[rl] - pbase) * 4, eb = (P[rl + 1] - pbase) * 4;
    float4 acc = f4z();
    // slots past the segment read the zero row through an ADDRESS select (+0.0f leaves the sum,
    // which starts at +0.0f, bit-identical), so the group's reads issue back to back
    for (int32_t kb = bb; kb < eb; kb += 4 * kUGroup) {
      float4 x[kUGroup];
#pragma unroll
      for (int q = 0; q < kUGroup; ++q) {
        const int32_t off = *reinterpret_cast<const int32_t*>(cb + ((kb + 4 * q < eb) ? kb + 4 * q : zb));
        x[q] = *reinterpret_cast<const float4*>(xb + off + ub);
      }
#pragma unroll
      for (int q = 0; q < kUGroup; ++q) f4acc(acc, x[q]);
    }
    if (pre) {
      finish_pre(a, r, c, q0, q1, acc);
    } else {
      finish_unit(a, r, c, acc);
    }
  }
}

// One tile of rows [r0, r0 + nr) whose row pointers P[0..nr] are in LDS, one column slice. spec: the
// tile is segment-aligned (whole molecules), so its own rows are staged while the first col piece
// loads. A tile whose col slice overflows the col_cap LDS slots runs in row pieces that fit, all
// summed from the same staged source rows (a molecule's pieces share its rows; a piece whose sources
// leave the staged span restages). Called by the whole workgroup after the barrier that published P;
// leaves every LDS region except the row pointers reusable.
template <bool SRC_CHUNKED, bool ADDS>
__device__ __forceinline__ void tile(const UnalArgs& a, const int32_t* P, int32_t* s_misc, int32_t* s_col, float* s_x,
                                     uint32_t r0, uint32_t nr, bool spec, uint32_t u0, const FastDiv& cs) {
  const int32_t base = P[0];
  if (P[nr] == base) {
    rows_global<SRC_CHUNKED>(a, P, nullptr, base, r0, nr, u0, cs);
    return;
  }
  const int32_t rb = (int32_t)(16 * a.pitch);  // bytes per staged row
  const char* xb = reinterpret_cast<const char*>(s_x);
  const char* cb = reinterpret_cast<const char*>(s_col);
  bool have = spec && nr + 1 <= a.xcap;  // s_x holds rows [first, first + span)
  uint32_t first = r0, span = nr;
  bool staging = have;  // the speculative stage is issued with the first piece's col loads
  for (uint32_t pr = 0; pr < nr;) {
    // rows [pr, pe) of the tile: the longest run from pr whose col entries fit (plus the sentinel)
    uint32_t pe = nr;
    while (pe > pr + 1 && (uint32_t)(P[pe] - P[pr]) >= a.col_cap) pe = pr + (pe - pr) / 2;
    const int32_t pb = P[pr] - base;
    const int32_t ncols = P[pe] - P[pr];
    if ((uint32_t)ncols >= a.col_cap) {  // one row longer than the slots: from global
      rows_global<SRC_CHUNKED>(a, P + pr, a.col + base + pb, base + pb, r0 + pr, pe - pr, u0, cs);
      pr = pe;
      continue;
    }
    int32_t lo = INT_MAX, hi = INT_MIN;
    // the col slice in batches of kCB loads per thread; with the speculative stage, each col batch
    // goes out together with a stage batch (one round trip for both)
    const bool spec_now = AIMX_HOPU_COMB && staging && a.D >= 4;
    const uint32_t sunits = spec_now ? span * cs.d : 0;
    const uint32_t ws = 4 * a.pitch;
    if (spec_now)
      for (uint32_t t = threadIdx.x; t < a.pitch; t += kUT) reinterpret_cast<float4*>(s_x + span * ws)[t] = f4z();
    for (uint32_t k = 0; (int32_t)(k * kCB * kUT) < ncols || k * kSB * kUT < sunits; ++k) {
      const int32_t i0 = (int32_t)(k * kCB * kUT);
      const uint32_t t0 = k * kSB * kUT;
      const bool cb_on = i0 < ncols, sb_on = t0 < sunits;  // workgroup-uniform
      int32_t c[kCB];
      float4 v[kSB];
      if (cb_on) {
#pragma unroll
        for (int b = 0; b < kCB; ++b) c[b] = a.col[base + pb + min(i0 + (int32_t)threadIdx.x + b * kUT, ncols - 1)];
      }
      if (sb_on) {
#pragma unroll
        for (int b = 0; b < kSB; ++b) {
          const uint32_t t = min(t0 + threadIdx.x + (uint32_t)b * kUT, sunits - 1);
          const uint32_t rl = fdiv(t, cs);
          v[b] = ld_raw(src_row<SRC_CHUNKED>(a, first + rl), 4 * (u0 + t - rl * cs.d), a.D);
        }
      }
      if (cb_on) {
#pragma unroll
        for (int b = 0; b < kCB; ++b) hold(c[b]);
#pragma unroll
        for (int b = 0; b < kCB; ++b) {
          const int32_t i = i0 + (int32_t)threadIdx.x + b * kUT;
          if (i < ncols) {
            s_col[i] = c[b];
            lo = min(lo, c[b]);
            hi = max(hi, c[b]);
          }
        }
      }
      if (sb_on) {
#pragma unroll
        for (int b = 0; b < kSB; ++b) hold(v[b]);
#pragma unroll
        for (int b = 0; b < kSB; ++b) {
          const uint32_t t = t0 + threadIdx.x + (uint32_t)b * kUT;
          if (t < sunits) {
            const uint32_t rl = fdiv(t, cs);
            put_raw(s_x + rl * ws, 4 * (u0 + t - rl * cs.d), a.D, u0, v[b]);
          }
        }
      }
    }
    if (staging && !spec_now) stage<SRC_CHUNKED>(a, s_x, first, span, u0, cs, a.pitch, false);
    staging = false;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, 64));
      hi = max(hi, __shfl_xor(hi, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
      atomicMin(&s_misc[2], lo);
      atomicMax(&s_misc[3], hi);
    }
    lds_barrier();
    lo = s_misc[2];
    hi = s_misc[3];
    if (!(have && lo >= (int32_t)first && hi < (int32_t)(first + span))) {
      if ((uint32_t)(hi - lo) + 1 >= a.xcap) {
        // sources too far apart to stage the whole slice: narrower sub-slices of the span that fit
        lds_barrier();  // every lo / hi read before the reset below
        if (threadIdx.x == 0) {
          s_misc[2] = INT_MAX;
          s_misc[3] = INT_MIN;
        }
        const uint32_t sp = (uint32_t)(hi - lo) + 1;
        const uint32_t su = min(cs.d, a.xcap * a.pitch / (sp + 1));  // units per sub-slice
        if (su == 0) {  // not even one unit of the span fits: from global
          rows_global<SRC_CHUNKED>(a, P + pr, s_col, base + pb, r0 + pr, pe - pr, u0, cs);
        } else {
          for (int32_t i = threadIdx.x; i < ncols; i += kUT) s_col[i] = (s_col[i] - lo) * (int32_t)(16 * su);
          if (threadIdx.x == 0) s_col[ncols] = (int32_t)(sp * 16 * su);
          for (uint32_t j0 = 0; j0 < cs.d; j0 += su) {
            const FastDiv fw = fastdiv_dev(min(su, cs.d - j0));
            stage<SRC_CHUNKED>(a, s_x, (uint32_t)lo, sp, u0 + j0, fw, su, true);
            lds_barrier();
            sum_rows<ADDS>(a, P + pr, P[pr], cb, xb, ncols * 4, r0 + pr, pe - pr, u0 + j0, fw, true);
            lds_barrier();  // staged rows read before the next sub-slice restages
          }
        }
        lds_barrier();  // s_col read before the next piece rewrites it
        have = false;   // s_x no longer holds a whole-slice stage
        pr = pe;
        continue;
      }
      // (the barrier above ordered every earlier stage write and staged-row read before this)
      first = (uint32_t)lo;
      span = (uint32_t)(hi - lo + 1);
      have = true;
      stage<SRC_CHUNKED>(a, s_x, first, span, u0, cs, a.pitch, false);
    }
    // col entries as byte offsets of the staged rows; each thread rewrites the entries it stored
    for (int32_t i = threadIdx.x; i < ncols; i += kUT) s_col[i] = (s_col[i] - (int32_t)first) * rb;
    if (threadIdx.x == 0) s_col[ncols] = (int32_t)span * rb;
    lds_barrier();
    if (threadIdx.x == 0) {  // every lo / hi read is behind the barrier above
      s_misc[2] = INT_MAX;
      s_misc[3] = INT_MIN;
    }
    sum_rows<ADDS>(a, P + pr, P[pr], cb, xb, ncols * 4, r0 + pr, pe - pr, u0, cs, a.compact);
    pr = pe;
    if (pr < nr) lds_barrier();  // s_col (and a restage of s_x) are rewritten by the next piece
  }
}

// Big tile bbig of the rows [split, rows) (hop chunks >= 1): skipped (skip_tail), a streaming zero
// fill, the residual terms alone, or (general CSR inputs only) a gather from global. Called by the
// whole workgroup; s_ptr / s_misc are scratch; ends with every LDS read done.
template <bool SRC_CHUNKED>
__device__ __forceinline__ void big_tile(const UnalArgs& a, uint32_t bbig, int32_t* s_ptr, int32_t* s_misc) {
  const uint32_t R0 = a.split + bbig * a.big_rows;
  const uint32_t NR = min(a.big_rows, a.rows - R0);
  if (threadIdx.x == 0) {
    s_misc[0] = a.rowptr[R0];
    s_misc[1] = a.rowptr[R0 + NR];
    // skip_tail: no edge from the start of R0's chunk to the end (every consumer trims those chunks)
    s_misc[2] = a.skip_tail && a.out_rpc.d > 0 && a.rowptr[fdiv(R0, a.out_rpc) * a.out_rpc.d] == a.rowptr[a.rows];
  }
  lds_barrier();
  const bool skip = s_misc[2] != 0, empty = s_misc[0] == s_misc[1];
  lds_barrier();  // s_misc is scratch again for the caller
  if (skip) return;
  if (empty) {
    if (a.flat_zero) {
      // the big tile's rows are one contiguous [NR, D] region: dword head, aligned float4 body, tail
      float* o = a.out + row_off(R0, a.out_ld, a.out_rpc, a.out_cs);
      const uint32_t n = NR * a.D;
      const uint32_t head = min(n, (uint32_t)((4u - (((uintptr_t)o >> 2) & 3u)) & 3u));
      if (threadIdx.x < head) o[threadIdx.x] = 0.f;
      const uint32_t body = (n - head) / 4;
      float4* ob = reinterpret_cast<float4*>(o + head);
      for (uint32_t t = threadIdx.x; t < body; t += kUT) ob[t] = f4z();
      const uint32_t tail = (n - head) - 4 * body;
      if (threadIdx.x < tail) o[head + 4 * body + threadIdx.x] = 0.f;
      return;
    }
    rows_global<SRC_CHUNKED>(a, nullptr, nullptr, 0, R0, NR, 0, a.upr_f);
    return;
  }
  // a big tile with edges (general CSR inputs only): its rows in tiles of tile_rows, whole width
  for (uint32_t r0 = R0; r0 < R0 + NR; r0 += a.tile_rows) {
    const uint32_t nr = min(a.tile_rows, R0 + NR - r0);
    for (uint32_t t = threadIdx.x; t <= nr; t += kUT) s_ptr[t] = a.rowptr[r0 + t];
    if (threadIdx.x == 0) {
      s_misc[2] = INT_MAX;
      s_misc[3] = INT_MIN;
    }
    lds_barrier();
    const int32_t base = s_ptr[0];
    rows_global<SRC_CHUNKED>(a, s_ptr, a.col + base, base, r0, nr, 0, a.upr_f);
    lds_barrier();
  }
}

template <bool SRC_CHUNKED, bool ADDS>
__global__ __launch_bounds__(kUT) void k_gather_unal(const UnalArgs a) {
  // [row pointers | misc | pad] [col_cap col entries] [xcap staged rows of 4 * cu floats]
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  int32_t* s_ptr = s_dyn;
  int32_t* s_misc = s_dyn + kUMisc;
  int32_t* s_col = s_dyn + kUHead;
  float* s_x = reinterpret_cast<float*>(s_dyn + kUHead + a.col_cap);
  // block order: big (zero-fill) tiles spread evenly among the tile workgroups (hop.hip)
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
  if (threadIdx.x == 0) {
    s_misc[2] = INT_MAX;
    s_misc[3] = INT_MIN;
  }
  if (is_small) {
    // the slices of one tile on one XCD: small blocks b and b + 8 k share an XCD (round-robin
    // dispatch), so tile = (b / (8 S)) * 8 + b % 8, slice = (b / 8) % S
    const uint32_t S = a.slices;
    const uint32_t grp = bsmall / (8 * S), in = bsmall - grp * 8 * S;
    const uint32_t ti = grp * 8 + (in & 7), sl = in >> 3;
    if (ti >= a.ntiles) return;
    const FastDiv cs = sl + 1 == S ? a.cu_last : a.cu_full;
    const uint32_t u0 = sl * a.cu;
    const uint32_t c0 = ti * a.tile_rows;
    const uint32_t c1 = min(c0 + a.tile_rows, a.split);
    if (!a.seg) {
      for (uint32_t t = threadIdx.x; t <= c1 - c0; t += kUT) s_ptr[t] = a.rowptr[c0 + t];
      lds_barrier();
      tile<SRC_CHUNKED, ADDS>(a, s_ptr, s_misc, s_col, s_x, c0, c1 - c0, false, u0, cs);
      return;
    }
    // segment-aligned cuts: each nominal cut c moves to the first molecule start in [c, c + 64) (c
    // itself if none); both cuts are the same function of c, so the tiles partition the rows
    const uint32_t pend = min(c1 + (uint32_t)kUAlignWin, a.split);
    for (uint32_t t = threadIdx.x; t <= pend - c0; t += kUT) s_ptr[t] = a.rowptr[c0 + t];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w < 2) {
      const uint32_t c = w ? c1 : c0;
      uint32_t cut = c;
      if (c > 0 && c < a.split) {
        const uint32_t q = min(c + lane, a.split - 1);
        const int64_t sq = a.seg[(int64_t)q * a.seg_stride], sp = a.seg[(int64_t)(q - 1) * a.seg_stride];
        const unsigned long long m = __ballot((c + lane < a.split) && sq != sp);
        if (m) cut = c + (uint32_t)__builtin_ctzll(m);
      }
      if (lane == 0) s_misc[w] = (int32_t)cut;
    }
    lds_barrier();
    const uint32_t r0 = (uint32_t)s_misc[0], r1 = (uint32_t)s_misc[1];
    if (r1 <= r0) return;
    tile<SRC_CHUNKED, ADDS>(a, s_ptr + (r0 - c0), s_misc, s_col, s_x, r0, r1 - r0, true, u0, cs);
    return;
  }
  big_tile<SRC_CHUNKED>(a, bbig, s_ptr, s_misc);
}



}  // namespace


int launch_gather_unal(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out, int64_t out_ld,
                       int64_t out_rpc, int64_t out_cs, const float* add0, int64_t add0_ld, const float* add1,
                       int64_t add1_ld, const int64_t* row_seg, int64_t row_seg_stride, hipStream_t stream,
                       int32_t skip_tail) {
  auto al4 = [](const void* p) { return ((uintptr_t)p & 3) == 0; };
  if (!al4(src) || !al4(out) || (add0 && !al4(add0)) || (add1 && !al4(add1))) return AIMX_EARG;
  if (rows >= (int64_t)INT32_MAX || src_rpc >= INT32_MAX || out_rpc >= INT32_MAX) return AIMX_EARG;
  // knobs, read once per process
  // slice width (floats): 64 = one 16-unit pitch per staged row (conflict-free ds_read_b128, sum_rows)
  static const int64_t w_max = std::max<int64_t>(4, tune_i64("AIMX_HOPU_W", 80) / 4 * 4);
  static const int64_t pitch_env = [] {  // staged row pitch in units: 0 compact, else a power of two >= 16
    const int64_t e = tune_i64("AIMX_HOPU_PITCH", 0);
    if (!e) return (int64_t)0;
    int64_t p = 16;
    while (p < e) p *= 2;
    return p;
  }();
  static const int64_t tr_env = std::max<int64_t>(1, std::min<int64_t>(kUMaxTile, tune_i64("AIMX_HOPU_TILE", 32)));
  static const int64_t col_cap_env = (std::max<int64_t>(64, tune_i64("AIMX_HOPU_COL_CAP", 1024)) + 3) / 4 * 4;
  static const int64_t stage_env = std::max<int64_t>(1024, tune_i64("AIMX_HOPU_STAGE", 20 * 1024));
  static const int64_t big_env = tune_i64("AIMX_HOPU_BIG", 256);
  static const int32_t interleave = tune_i64("AIMX_HOP_INTERLEAVE", 1) != 0 ? 1 : 0;
  static const bool no_seg = tune_i64("AIMX_HOP_NO_SEG", 0) != 0;
  const int64_t upr = cdiv(D, 4);
  // slices of cu units; the last slice must hold more than a partial last unit (put_raw writes that
  // unit shifted down over the unit before it, which must be in the same slice)
  // (the requested count s grows monotonically — the realised count cdiv(upr, cu) may be smaller,
  // so stepping that instead could revisit the same split forever — and a split never found ends
  // at one slice, which always qualifies)
  int64_t slices = 1, cu = upr, cu_last = upr;
  for (int64_t s = cdiv(upr * 4, w_max); s > 1 && s <= upr; ++s) {
    const int64_t c = cdiv(upr, s), n = cdiv(upr, c), last = upr - (n - 1) * c;
    if (D % 4 == 0 || D < 4 || n == 1 || last >= 2) {
      slices = n;
      cu = c;
      cu_last = last;
      break;
    }
  }
  if (cu_last <= 0) return AIMX_EARG;
  const int64_t split = (out_rpc > 0 && out_rpc < rows) ? out_rpc : rows;
  // with few tiles (small batches) shorter nominal tiles keep the CUs busy
  int64_t tr = tr_env;
  while (tr > 8 && cdiv(split, tr) * slices < 2048) tr /= 2;
  const int64_t ntiles = cdiv(split, tr);
  const int64_t nsmall = cdiv(ntiles, 8) * 8 * slices;  // whole groups of 8 tiles (XCD order)
  const int64_t big = std::max<int64_t>(tr, big_env);
  const int64_t nbig = cdiv(rows - split, big);
  int64_t pitch = pitch_env;
  while (pitch_env && pitch < cu) pitch *= 2;
  if (!pitch_env) pitch = cu;  // compact: no idle lanes, rows of cu units
  int64_t pitch_l2 = 0;
  while (pitch_env && (1ll << pitch_l2) < pitch) ++pitch_l2;
  const int64_t xcap = std::min<int64_t>(kUMaxRows + 1, stage_env / (16 * pitch));
  const size_t dyn = (size_t)(kUHead + col_cap_env) * 4 + (size_t)xcap * 16 * pitch;
  UnalArgs a;
  a.src = src;
  a.src_ld = src_ld;
  a.src_cs = src_cs;
  a.src_rpc = make_fastdiv(src_rpc > 0 ? (uint32_t)src_rpc : 0);
  a.rowptr = rowptr;
  a.col = col;
  a.D = (uint32_t)D;
  a.upr = (uint32_t)upr;
  a.slices = (uint32_t)slices;
  a.cu = (uint32_t)cu;
  a.pitch = (uint32_t)pitch;
  a.pitch_l2 = (uint32_t)pitch_l2;
  a.compact = pitch_env ? 0 : 1;
  a.cu_full = make_fastdiv((uint32_t)cu);
  a.cu_last = make_fastdiv((uint32_t)cu_last);
  a.upr_f = make_fastdiv((uint32_t)upr);
  a.rows = (uint32_t)rows;
  a.split = (uint32_t)split;
  a.tile_rows = (uint32_t)tr;
  a.ntiles = (uint32_t)ntiles;
  a.nsmall = (uint32_t)nsmall;
  a.big_rows = (uint32_t)big;
  a.nbig = (uint32_t)nbig;
  a.col_cap = (uint32_t)col_cap_env;
  a.xcap = (uint32_t)xcap;
  a.out = out;
  a.out_ld = out_ld;
  a.out_cs = out_cs;
  a.out_rpc = make_fastdiv(out_rpc > 0 ? (uint32_t)out_rpc : 0);
  a.add0 = add0;
  a.add0_ld = add0_ld;
  a.add1 = add1;
  a.add1_ld = add1_ld;
  a.seg = (row_seg && !no_seg) ? row_seg : nullptr;
  a.q0 = add0 ? add0 : src;
  a.q0_ld = add0 ? add0_ld : 0;
  a.q1 = add1 ? add1 : src;
  a.q1_ld = add1 ? add1_ld : 0;
  a.seg_stride = row_seg_stride;
  const bool contiguous = out_ld == D && (out_rpc <= 0 || out_cs == out_rpc * out_ld);
  a.flat_zero = (contiguous && !add0 && !add1) ? 1 : 0;
  a.interleave = interleave;
  a.skip_tail = skip_tail;
  const int64_t blocks = nsmall + nbig;
  if (blocks <= 0) return AIMX_OK;
  if (blocks >= (int64_t)INT32_MAX) return AIMX_EARG;
  using KFn = void (*)(const UnalArgs);
  const bool adds = D >= 4 && (add0 || add1);
  KFn fn = src_rpc > 0 ? (adds ? k_gather_unal<true, true> : k_gather_unal<true, false>)
                       : (adds ? k_gather_unal<false, true> : k_gather_unal<false, false>);
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kUT), dyn, stream, a);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

}  // namespace aimx
