// The hop for rows that are not runs of 16-byte vectors: the odd widths D = int(0.3 * hidden)
// (153 / 307 at hidden 512 / 1024, reference src/models/gnn.py:100) and rows that start at
// unaligned addresses (a hop chunk of the concatenated [x | chunk_0 | ...] matrix sits at column
// offset D, layers.py:76-79). Same contract and bit-exact result as hop.hip (the ordered edge-order
// sum of CPU scatter_add_, layers.py:133-167); hop.hip keeps the 16-byte-aligned rows.
//
// Every global access of x and of the output is an aligned 16-byte vector; the alignment is fixed
// up in LDS, one column pass (<= 80 floats of every row) at a time:
//   1. stage: each source row the tile reads is fetched as the aligned float4 run that covers the
//      pass's columns and written to LDS at a 16-byte-aligned row start (column c at s_x[row*wc+c]);
//   2. sum: each thread owns normalized units (row, 4 columns) and sums the staged rows of the row's
//      CSR segment with ds_read_b128 (zero-row padding and an address select, as in hop.hip),
//      results in registers;
//   3. shift: the results go back to LDS in the OUTPUT row's alignment (column c of row r at
//      s_x[r * (wc + 4) + mis(r) + c], mis = the row start's float offset inside its 16 bytes);
//   4. store: aligned float4 stores of every whole unit; only the partial units at a row's (or a
//      pass's) ends take dword stores. The residual terms of the backward are added here.
// Tiles are molecules: a workgroup owns the molecules that START in its window of `win` rows
// (molecule starts found from the batch indices with one ballot per 64 rows), so a tile's sources
// are its own rows and x is staged once. A molecule whose pair list overflows the LDS col slots is
// cut into pieces that fit (restaged per piece). For small (latency-bound) batches the column
// passes of a window run in separate workgroups (pass split). The zero hop chunks (the reference's
// chunks >= 1 are empty: targets are never hop-offset, layers.py:154 / molecular.py:426-436) are
// streaming aligned stores in big tiles spread among the molecule tiles.
//
// Measured alternatives (round 3, profiles/r03_hop_rows_ab.txt): a software pipeline that loads the
// next item while the current one is summed, narrower passes with a separate output tile, and a
// register realignment by lane shuffle (no output tile) all ran slower at the c4 / c5 roofline size.
// Round 4: one wave per output row reading every source row straight from L1 / L2 (no LDS) was
// 7-13 % faster in the step (c5 hop forward 54.5 -> 47.6 us) but 1.3-1.7x slower at the roofline
// size, where it is bound by L2 bandwidth (each source row is re-read once per pair: E / N = 11-31).
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "aimx_common.h"
#include "hop_common.h"

namespace aimx {
namespace {

constexpr int kRT = 256;      // threads per workgroup
constexpr int kRMaxU = 6;     // normalized units (4 columns of a row) per thread per pass, in registers
constexpr int kRScan = 128;   // rows whose row pointers and molecule starts one round trip loads
constexpr int kRMisc = 132;   // int offset of the misc words: [0] lo, [1] hi, [2..5] start mask (4 x 32 bits)
constexpr int kRHead = 144;   // ints ahead of the col slice (row pointers [129] + misc), 16-byte multiple

struct RowsArgs {
  const float* src;
  int64_t src_ld, src_cs;
  FastDiv src_rpc;
  const int32_t* rowptr;
  const int32_t* col;
  uint32_t D, wc, passes;     // row width; pass width (floats, multiple of 4); ceil(D / wc)
  FastDiv wu_full, wu_last;   // normalized units per row in a full pass / the last pass
  FastDiv uo_full, uo_last;   // output (and staging) units per row: one more, for the misalignment
  FastDiv uo_row;             // output units of a whole row (zero rows)
  uint32_t rows, split;       // windows cover rows [0, split); big tiles rows [split, rows)
  uint32_t win, nwin, cap, col_cap;
  uint32_t pass_split;        // each window's passes in separate workgroups
  uint32_t nsmall;            // window workgroups: nwin (x passes with pass_split)
  uint32_t big_rows, nbig;
  int32_t interleave, flat_zero;
  float* out;
  int64_t out_ld, out_cs;
  FastDiv out_rpc;
  const float* add0;
  int64_t add0_ld;
  int32_t add0_early;  // every add0 row starts 16-byte aligned: added in the sum phase
  const float* add1;
  int64_t add1_ld;
  const int64_t* seg;  // molecule id per row of [0, split) (optional)
  int64_t seg_stride;
  int32_t lean;  // fewer barriers per piece (AIMX_HOPR_LEAN=0: the round-3 schedule, for A/B)
  int32_t skip_tail;  // big tiles in the trailing EMPTY hop chunks are not written (segment_gather_sum)
};

__device__ __forceinline__ uint32_t misal(const void* p) { return (uint32_t)((uintptr_t)p >> 2) & 3u; }

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ float4 f4add(const float4& a, const float4& b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <bool SRC_CHUNKED>
__device__ __forceinline__ const float* src_row(const RowsArgs& a, uint32_t q) {
  if (!SRC_CHUNKED) return a.src + (int64_t)q * a.src_ld;
  const uint32_t k = fdiv(q, a.src_rpc);
  return a.src + (int64_t)(q - k * a.src_rpc.d) * a.src_ld + (int64_t)k * a.src_cs;
}

__device__ __forceinline__ float* out_row(const RowsArgs& a, uint32_t r) {
  return a.out + row_off(r, a.out_ld, a.out_rpc, a.out_cs);
}

// Column pass p: first column, width, units per row (normalized / output).
struct Pass {
  uint32_t c0, w;
  FastDiv wu, uo;
};
__device__ __forceinline__ FastDiv fd_sel(bool c, const FastDiv& x, const FastDiv& y) {
  // field by field: a select of whole structs becomes a private-memory copy
  return FastDiv{c ? x.d : y.d, c ? x.m : y.m, c ? x.l : y.l};
}
__device__ __forceinline__ Pass pass_of(const RowsArgs& a, uint32_t p) {
  const bool last = p + 1 == a.passes;
  return Pass{p * a.wc, last ? a.D - p * a.wc : a.wc, fd_sel(last, a.wu_last, a.wu_full),
              fd_sel(last, a.uo_last, a.uo_full)};
}

// Rows [first, first + span), columns [c0, c0 + w) of src -> s_x (row stride wc, 16-byte-aligned
// rows), plus an all-zero row at index span. Each source row is read as the aligned float4 run
// covering it (at most 3 floats past either end, inside the same 16 bytes: never a fault).
template <bool SRC_CHUNKED>
__device__ __forceinline__ void stage_rows(const RowsArgs& a, float* s_x, uint32_t first, uint32_t span,
                                           const Pass& ps) {
  const FastDiv& su = ps.uo;
  const uint32_t units = span * su.d;
  const int32_t wi = (int32_t)ps.w;
  for (uint32_t t = threadIdx.x; t < units; t += kRT) {
    const uint32_t rl = fdiv(t, su);
    const uint32_t k = t - rl * su.d;
    const float* g = src_row<SRC_CHUNKED>(a, first + rl) + ps.c0;
    const uint32_t m = misal(g);
    const int32_t c = (int32_t)(4 * k) - (int32_t)m;  // column of v.x (> -4)
    if (c >= wi) continue;
    const float4 v = *reinterpret_cast<const float4*>(g - m + 4 * k);
    float* d = s_x + rl * a.wc;
    if (m == 0 && c + 3 < wi) {
      *reinterpret_cast<float4*>(d + c) = v;
    } else {
      if (c >= 0) d[c] = v.x;
      if (c + 1 >= 0 && c + 1 < wi) d[c + 1] = v.y;
      if (c + 2 >= 0 && c + 2 < wi) d[c + 2] = v.z;
      if (c + 3 < wi) d[c + 3] = v.w;
    }
  }
  float4* z = reinterpret_cast<float4*>(s_x + span * a.wc);
  for (uint32_t t = threadIdx.x; t < a.wc / 4; t += kRT) z[t] = f4zero();
}

// stage_rows in two halves: the aligned float4 loads into registers (at most kRMaxU per thread;
// the caller checks span * uo <= kRMaxU * kRT), and later their LDS stores plus the zero row. The
// loads of the next column pass are issued before this pass's output stores, so their round trip
// overlaps the stores instead of following the barrier after them.
template <bool SRC_CHUNKED>
__device__ __forceinline__ void stage_load(const RowsArgs& a, float4 (&v)[kRMaxU], uint32_t first, uint32_t span,
                                           const Pass& ps) {
  const uint32_t units = span * ps.uo.d;
#pragma unroll
  for (int j = 0; j < kRMaxU; ++j) {
    const uint32_t t = threadIdx.x + (uint32_t)j * kRT;
    v[j] = f4zero();  // written on every path: the registers carry nothing across passes
    if (t < units) {
      const uint32_t rl = fdiv(t, ps.uo);
      const uint32_t k = t - rl * ps.uo.d;
      const float* g = src_row<SRC_CHUNKED>(a, first + rl) + ps.c0;
      const uint32_t m = misal(g);
      if ((int32_t)(4 * k) - (int32_t)m < (int32_t)ps.w) v[j] = *reinterpret_cast<const float4*>(g - m + 4 * k);
    }
  }
}
template <bool SRC_CHUNKED>
__device__ __forceinline__ void stage_put(const RowsArgs& a, float* s_x, const float4 (&v)[kRMaxU], uint32_t first,
                                          uint32_t span, const Pass& ps) {
  const uint32_t units = span * ps.uo.d;
  const int32_t wi = (int32_t)ps.w;
#pragma unroll
  for (int j = 0; j < kRMaxU; ++j) {
    const uint32_t t = threadIdx.x + (uint32_t)j * kRT;
    if (t < units) {
      const uint32_t rl = fdiv(t, ps.uo);
      const uint32_t k = t - rl * ps.uo.d;
      const uint32_t m = misal(src_row<SRC_CHUNKED>(a, first + rl) + ps.c0);
      const int32_t c = (int32_t)(4 * k) - (int32_t)m;
      if (c >= wi) continue;
      float* d = s_x + rl * a.wc;
      if (m == 0 && c + 3 < wi) {
        *reinterpret_cast<float4*>(d + c) = v[j];
      } else {
        if (c >= 0) d[c] = v[j].x;
        if (c + 1 >= 0 && c + 1 < wi) d[c + 1] = v[j].y;
        if (c + 2 >= 0 && c + 2 < wi) d[c + 2] = v[j].z;
        if (c + 3 < wi) d[c + 3] = v[j].w;
      }
    }
  }
  float4* z = reinterpret_cast<float4*>(s_x + span * a.wc);
  for (uint32_t t = threadIdx.x; t < a.wc / 4; t += kRT) z[t] = f4zero();
}

// v (columns c .. c+3 of a row, c = 4u - m) += the same columns of row `arow` (pass-relative base).
// first: v = add + v (the order hop.hip uses for add0), else v = v + add.
__device__ __forceinline__ void add_cols(float4& v, const float* arow, uint32_t m, uint32_t u, int32_t c, int32_t w,
                                         bool first) {
  float4 s;
  if (misal(arow) == m) {
    s = *reinterpret_cast<const float4*>(arow - m + 4 * u);
  } else {
    s.x = (c >= 0) ? arow[c] : 0.f;
    s.y = (c + 1 >= 0 && c + 1 < w) ? arow[c + 1] : 0.f;
    s.z = (c + 2 >= 0 && c + 2 < w) ? arow[c + 2] : 0.f;
    s.w = (c + 3 < w) ? arow[c + 3] : 0.f;
  }
  v = first ? f4add(s, v) : f4add(v, s);
}

// Output unit of a row: an aligned float4 store when all 4 columns are the row's, else dwords.
__device__ __forceinline__ void store_unit(float* og, const float4& v, int32_t c, int32_t w) {
  if (c >= 0 && c + 3 < w) {
    *reinterpret_cast<float4*>(og) = v;
  } else {
    if (c >= 0) og[0] = v.x;
    if (c + 1 >= 0 && c + 1 < w) og[1] = v.y;
    if (c + 2 >= 0 && c + 2 < w) og[2] = v.z;
    if (c + 3 < w) og[3] = v.w;
  }
}

// Zero columns [c0, c0 + w) of rows [r0, r0 + nr) (no residual terms): aligned stores, no LDS.
__device__ __forceinline__ void zero_rows(const RowsArgs& a, uint32_t r0, uint32_t nr, uint32_t c0, uint32_t w,
                                          const FastDiv& uo) {
  const uint32_t units = nr * uo.d;
  for (uint32_t t = threadIdx.x; t < units; t += kRT) {
    const uint32_t rl = fdiv(t, uo);
    const uint32_t u = t - rl * uo.d;
    float* o = out_row(a, r0 + rl) + c0;
    const uint32_t m = misal(o);
    const int32_t c = (int32_t)(4 * u) - (int32_t)m;
    if (c >= (int32_t)w) continue;
    store_unit(o - m + 4 * u, f4zero(), c, (int32_t)w);
  }
}

// Normalized unit (row rl, columns 4v..) of a pass into the output tile, in the output row's
// alignment m (the 16-byte-aligned LDS positions are then the output's aligned units).
__device__ __forceinline__ void tile_put(float* s_t, uint32_t ot, uint32_t rl, uint32_t m, uint32_t v, int32_t lim,
                                         const float4& r) {
  float* d = s_t + rl * ot + m + 4 * v;
  if (lim >= 4 && m == 0) {
    *reinterpret_cast<float4*>(d) = r;
  } else if (lim >= 4 && m == 2) {
    reinterpret_cast<float2*>(d)[0] = make_float2(r.x, r.y);
    reinterpret_cast<float2*>(d)[1] = make_float2(r.z, r.w);
  } else if (lim >= 4) {  // m odd: d + 1 is 8-byte aligned
    d[0] = r.x;
    *reinterpret_cast<float2*>(d + 1) = make_float2(r.y, r.z);
    d[3] = r.w;
  } else {
    d[0] = r.x;
    if (lim > 1) d[1] = r.y;
    if (lim > 2) d[2] = r.z;
  }
}

// One piece of rows [r0, r0 + nr) (nr <= cap) whose row pointers are P[0..nr] in LDS, column passes
// [p0, p1). Called by the whole workgroup after a barrier; leaves every LDS region except the row
// pointers reusable. spec: the piece is (part of) a molecule, so its own rows are staged while
// the col slice loads.
template <bool SRC_CHUNKED, bool PRE>
__device__ __forceinline__ void piece(const RowsArgs& a, const int32_t* P, int32_t* s_misc, int32_t* s_col,
                                      float* s_x, uint32_t r0, uint32_t nr, bool spec, uint32_t p0, uint32_t p1) {
  const int32_t base = P[0];
  const int32_t ncols = P[nr] - base;
  const bool has_adds = a.add0 || a.add1;
  int mode = ncols == 0 ? 0 : ((uint32_t)ncols < a.col_cap ? 1 : 2);  // 0 no edges, 1 staged, 2 global
  uint32_t first = r0, span = nr;
  if (mode == 1) {
    const Pass ps = pass_of(a, p0);
    const int32_t rb = (int32_t)a.wc * 4;
    // lean: the lo / hi words were reset by scan_window or by the previous piece (after a barrier
    // that follows every read of them), and a molecule piece stores its col slice already as byte
    // offsets into its own staged rows, so the common case needs no barrier after the min / max
    const bool conv = a.lean && spec;
    if (!a.lean) {
      if (threadIdx.x == 0) {
        s_misc[0] = INT_MAX;
        s_misc[1] = INT_MIN;
      }
      __syncthreads();
    }
    int32_t lo = INT_MAX, hi = INT_MIN;
    for (int32_t i = threadIdx.x; i < ncols; i += kRT) {
      const int32_t c = a.col[base + i];
      // (wrapping arithmetic: an entry far outside the piece only matters if the piece is not its own
      // source span, and then the slice is re-read from global below)
      s_col[i] = conv ? (int32_t)((uint32_t)(c - (int32_t)r0) * (uint32_t)rb) : c;
      lo = min(lo, c);
      hi = max(hi, c);
    }
    if (conv && threadIdx.x == 0) s_col[ncols] = (int32_t)nr * rb;
    // a molecule tile's sources are its own rows: stage them while the col slice is in flight
    if (spec) stage_rows<SRC_CHUNKED>(a, s_x, r0, nr, ps);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, 64));
      hi = max(hi, __shfl_xor(hi, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
      atomicMin(&s_misc[0], lo);
      atomicMax(&s_misc[1], hi);
    }
    __syncthreads();
    lo = s_misc[0];
    hi = s_misc[1];
    bool sync = true;
    const bool own = spec && lo >= (int32_t)r0 && hi < (int32_t)(r0 + nr);
    if (own) {
      sync = !conv;  // staged: own rows (converted already under conv)
    } else if ((uint32_t)(hi - lo) < a.cap) {
      first = (uint32_t)lo;
      span = (uint32_t)(hi - lo + 1);
      stage_rows<SRC_CHUNKED>(a, s_x, first, span, ps);
    } else {
      mode = 2;  // s_col keeps the raw col slice
    }
    // each thread rewrites only the entries it stored itself; the sentinel is thread 0's
    if (mode == 1 && !conv) {
      for (int32_t i = threadIdx.x; i < ncols; i += kRT) s_col[i] = (s_col[i] - (int32_t)first) * rb;
      if (threadIdx.x == 0) s_col[ncols] = (int32_t)span * rb;
    } else if (mode == 1 && !own) {  // conv, restaged at [first, first + span): raw cols from global
      for (int32_t i = threadIdx.x; i < ncols; i += kRT) s_col[i] = (a.col[base + i] - (int32_t)first) * rb;
      if (threadIdx.x == 0) s_col[ncols] = (int32_t)span * rb;
    }  // mode 2 after conv reads the raw cols from global (col_raw below)
    if (sync) __syncthreads();
  }
  const char* xb = reinterpret_cast<const char*>(s_x);
  const char* cb = reinterpret_cast<const char*>(s_col);
  const uint32_t ot = a.wc + 4;
  float4 pre[kRMaxU];  // the next pass's staged rows (stage_load), when they fit
  bool pre_ok = false;
  for (uint32_t p = p0; p < p1; ++p) {
    const Pass ps = pass_of(a, p);
    const FastDiv& wu = ps.wu;
    const FastDiv& uo = ps.uo;
    if (mode == 0 && !has_adds) {
      zero_rows(a, r0, nr, ps.c0, ps.w, uo);
      continue;
    }
    if (p > p0 && mode == 1) {
      if (pre_ok)
        stage_put<SRC_CHUNKED>(a, s_x, pre, first, span, ps);
      else
        stage_rows<SRC_CHUNKED>(a, s_x, first, span, ps);
      __syncthreads();
    }
    // sum phase: normalized units (row rl, columns 4v..4v+3 of this pass), in registers
    const uint32_t units = nr * wu.d;
    float4 res[kRMaxU];
#pragma unroll
    for (int j = 0; j < kRMaxU; ++j) {
      const uint32_t t = threadIdx.x + (uint32_t)j * kRT;
      float4 acc = f4zero();
      if (t < units) {
        const uint32_t rl = fdiv(t, wu);
        const uint32_t v = t - rl * wu.d;
        if (mode == 1) {
          const uint32_t ub = v * 16;
          const int32_t zb = ncols * 4;
          const int32_t bb = (P[rl] - base) * 4, eb = (P[rl + 1] - base) * 4;
          // slots past the segment read the zero row: an ADDRESS select keeps the four slot reads
          // unpredicated, so they issue back to back (a value select becomes a branch per read)
          for (int32_t kb = bb; kb < eb; kb += 16) {
            float4 x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int32_t off = *reinterpret_cast<const int32_t*>(cb + ((kb + 4 * q < eb) ? kb + 4 * q : zb));
              x[q] = *reinterpret_cast<const float4*>(xb + off + ub);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) acc = f4add(acc, x[q]);
          }
        } else if (mode == 2) {
          // fallback (tile sources wider than the staging capacity, or an over-long col slice):
          // dword gathers from global, same order
          const int32_t b = P[rl] - base, e = P[rl + 1] - base;
          const int32_t* cols = ((uint32_t)ncols < a.col_cap && !(a.lean && spec)) ? s_col : a.col + base;
          const int32_t lim = (int32_t)ps.w - (int32_t)(4 * v);
          float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
          for (int32_t k = b; k < e; ++k) {
            const float* xr = src_row<SRC_CHUNKED>(a, (uint32_t)cols[k]) + ps.c0 + 4 * v;
            s0 += xr[0];
            if (lim > 1) s1 += xr[1];
            if (lim > 2) s2 += xr[2];
            if (lim > 3) s3 += xr[3];
          }
          acc = make_float4(s0, s1, s2, s3);
        }
        if (a.add0_early)
          acc = f4add(*reinterpret_cast<const float4*>(a.add0 + (int64_t)(r0 + rl) * a.add0_ld + ps.c0 + 4 * v), acc);
      }
      res[j] = acc;
    }
    __syncthreads();  // every staged row read: s_x becomes the output tile
    if (a.lean && p == p0 && threadIdx.x == 0) {  // every lo / hi read is behind this barrier
      s_misc[0] = INT_MAX;
      s_misc[1] = INT_MIN;
    }
#pragma unroll
    for (int j = 0; j < kRMaxU; ++j) {
      const uint32_t t = threadIdx.x + (uint32_t)j * kRT;
      if (t < units) {
        const uint32_t rl = fdiv(t, wu);
        const uint32_t v = t - rl * wu.d;
        tile_put(s_x, ot, rl, misal(out_row(a, r0 + rl)), v, (int32_t)ps.w - (int32_t)(4 * v), res[j]);
      }
    }
    __syncthreads();
    pre_ok = false;
    if (PRE && mode == 1 && p + 1 < p1) {
      const Pass pn = pass_of(a, p + 1);
      pre_ok = span * pn.uo.d <= (uint32_t)(kRMaxU * kRT);
      if (pre_ok) stage_load<SRC_CHUNKED>(a, pre, first, span, pn);
    }
    const uint32_t ounits = nr * uo.d;
    for (uint32_t t = threadIdx.x; t < ounits; t += kRT) {
      const uint32_t rl = fdiv(t, uo);
      const uint32_t u = t - rl * uo.d;
      const uint32_t r = r0 + rl;
      float* o = out_row(a, r) + ps.c0;
      const uint32_t m = misal(o);
      const int32_t c = (int32_t)(4 * u) - (int32_t)m;
      if (c >= (int32_t)ps.w) continue;
      float4 v = *reinterpret_cast<const float4*>(s_x + rl * ot + 4 * u);
      if (a.add0 && !a.add0_early) add_cols(v, a.add0 + (int64_t)r * a.add0_ld + ps.c0, m, u, c, (int32_t)ps.w, true);
      if (a.add1) add_cols(v, a.add1 + (int64_t)r * a.add1_ld + ps.c0, m, u, c, (int32_t)ps.w, false);
      store_unit(o - m + 4 * u, v, c, (int32_t)ps.w);
    }
    __syncthreads();
  }
}

// Row pointers of rows [pb, pb + pn] and (with_seg) the molecule-start bits of rows [pb, pb + pn)
// into LDS in one round trip, pn = min(kRScan, limit - pb); ends with a barrier.
__device__ __forceinline__ uint32_t scan_window(const RowsArgs& a, int32_t* s_ptr, int32_t* s_misc, uint32_t pb,
                                                uint32_t limit, bool with_seg) {
  const uint32_t pn = min((uint32_t)kRScan, limit - pb);
  for (uint32_t t = threadIdx.x; t <= pn; t += kRT) s_ptr[t] = a.rowptr[pb + t];
  if (a.lean && threadIdx.x == 0) {  // the next piece's col-slice min / max
    s_misc[0] = INT_MAX;
    s_misc[1] = INT_MIN;
  }
  if (with_seg && threadIdx.x < 128) {
    const uint32_t q = pb + threadIdx.x;
    bool st = false;
    if (threadIdx.x < pn) st = (q == 0) || a.seg[(int64_t)q * a.seg_stride] != a.seg[(int64_t)(q - 1) * a.seg_stride];
    const unsigned long long m = __ballot(st);
    if ((threadIdx.x & 63) == 0) {
      const int wv = threadIdx.x >> 6;
      s_misc[2 + 2 * wv] = (int32_t)(uint32_t)m;
      s_misc[3 + 2 * wv] = (int32_t)(uint32_t)(m >> 32);
    }
  }
  __syncthreads();
  return pn;
}

// First molecule start in [from, pb + pn) from the LDS start bits, or -1.
__device__ __forceinline__ int64_t next_start(const int32_t* s_misc, uint32_t pb, uint32_t pn, uint32_t from) {
  for (uint32_t i = from - pb; i < pn;) {
    const uint32_t wd = (uint32_t)s_misc[2 + (i >> 5)] >> (i & 31);
    if (wd) {
      const uint32_t j = i + (uint32_t)__builtin_ctz(wd);
      return j < pn ? (int64_t)(pb + j) : -1;
    }
    i = (i | 31) + 1;
  }
  return -1;
}

// PRE: the next column pass's staging loads are issued before this pass's stores (stage_load):
// 112 VGPRs (4 waves per SIMD) instead of 88 (5)
template <bool SRC_CHUNKED, bool PRE>
__global__ __launch_bounds__(kRT) void k_gather_rows(const RowsArgs a) {
  // [row pointers | misc | pad] [col_cap col entries] [staged rows / output tile]
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  int32_t* s_ptr = s_dyn;
  int32_t* s_misc = s_dyn + kRMisc;
  int32_t* s_col = s_dyn + kRHead;
  float* s_x = reinterpret_cast<float*>(s_dyn + kRHead + a.col_cap);
  // block order: big (zero-fill) tiles spread evenly among the window workgroups (hop.hip)
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
  uint32_t R0, R1, p0 = 0, p1 = a.passes;
  if (is_small) {
    uint32_t w = bsmall;
    if (a.pass_split) {
      w = bsmall / a.passes;
      p0 = bsmall - w * a.passes;
      p1 = p0 + 1;
    }
    R0 = w * a.win;
    R1 = min(R0 + a.win, a.split);
  } else {
    R0 = a.split + bbig * a.big_rows;
    R1 = min(R0 + a.big_rows, a.rows);
    if (threadIdx.x == 0) {
      s_misc[0] = a.rowptr[R0];
      s_misc[1] = a.rowptr[R1];
      // skip_tail: no edge from the start of R0's chunk to the end (every consumer trims those chunks)
      s_misc[2] = a.skip_tail && a.out_rpc.d > 0 &&
                  a.rowptr[fdiv(R0, a.out_rpc) * a.out_rpc.d] == a.rowptr[a.rows];
    }
    __syncthreads();
    if (s_misc[2]) return;
    const bool empty = s_misc[0] == s_misc[1];
    if (empty && a.flat_zero) {
      // the big tile's rows are one contiguous [NR, D] region: head dwords, aligned float4 body, tail
      float* o = out_row(a, R0);
      const uint32_t n = (R1 - R0) * a.D;
      const uint32_t head = min(n, (4u - misal(o)) & 3u);
      if (threadIdx.x < head) o[threadIdx.x] = 0.f;
      const uint32_t body = (n - head) / 4;
      float4* ob = reinterpret_cast<float4*>(o + head);
      for (uint32_t t = threadIdx.x; t < body; t += kRT) ob[t] = f4zero();
      const uint32_t tail = (n - head) - 4 * body;
      if (threadIdx.x < tail) o[head + 4 * body + threadIdx.x] = 0.f;
      return;
    }
    if (empty && !a.add0 && !a.add1) {
      zero_rows(a, R0, R1 - R0, 0, a.D, a.uo_row);
      return;
    }
    __syncthreads();
  }
  // Pieces: with molecule ids (window workgroups), the molecules that start in [R0, R1), each
  // whole; otherwise rows [R0, R1) in runs of cap; either way cut until the col slice fits.
  const bool seg = is_small && a.seg != nullptr;
  const uint32_t limit = seg ? a.split : R1;
  uint32_t pb = R0;
  uint32_t pn = scan_window(a, s_ptr, s_misc, pb, limit, seg);
  uint32_t m = R0;
  if (seg) {
    const int64_t s = next_start(s_misc, pb, pn, R0);
    if (s < 0 || (uint32_t)s >= R1) return;
    m = (uint32_t)s;
  }
  while (m < limit) {
    if (m >= pb + pn) {
      __syncthreads();  // the last piece's row pointers are read
      pb = m;
      pn = scan_window(a, s_ptr, s_misc, pb, limit, seg);
    }
    uint32_t end = pb + pn;
    if (seg) {
      if (m >= R1 && next_start(s_misc, pb, pn, m) == (int64_t)m) break;  // the next window's molecule
      const int64_t e = next_start(s_misc, pb, pn, m + 1);
      if (e >= 0) end = (uint32_t)e;
    }
    uint32_t pe = min(end, m + a.cap);
    while (pe > m + 1 && (uint32_t)(s_ptr[pe - pb] - s_ptr[m - pb]) >= a.col_cap) pe = m + (pe - m) / 2;
    piece<SRC_CHUNKED, PRE>(a, s_ptr + (m - pb), s_misc, s_col, s_x, m, pe - m, seg, p0, p1);
    m = pe;
  }
}

int64_t env_i64(const char* name, int64_t dflt) {
  const char* e = getenv(name);
  return e ? std::max<int64_t>(0, atoll(e)) : dflt;
}

}  // namespace

int launch_gather_rows(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out, int64_t out_ld,
                       int64_t out_rpc, int64_t out_cs, const float* add0, int64_t add0_ld, const float* add1,
                       int64_t add1_ld, const int64_t* row_seg, int64_t row_seg_stride, hipStream_t stream,
                       int32_t skip_tail, bool windows) {
  // 4-byte-aligned fp32 rows (the 16-byte fix-up works on float offsets)
  auto al4 = [](const void* p) { return ((uintptr_t)p & 3) == 0; };
  if (!al4(src) || !al4(out) || (add0 && !al4(add0)) || (add1 && !al4(add1))) return AIMX_EARG;
  if (rows >= (int64_t)INT32_MAX || src_rpc >= INT32_MAX || out_rpc >= INT32_MAX) return AIMX_EARG;
  // knobs, read once per process (no per-launch getenv)
  static const int64_t wc_max = std::max<int64_t>(4, env_i64("AIMX_HOPR_WC", 80) / 4 * 4);
  static const int64_t cap_env = std::max<int64_t>(8, env_i64("AIMX_HOPR_CAP", 64));
  static const int64_t col_cap = (std::max<int64_t>(64, env_i64("AIMX_HOPR_COL_CAP", 2048)) + 3) / 4 * 4;
  static const int64_t win_env = env_i64("AIMX_HOPR_WIN", 32);
  static const int64_t big_env = env_i64("AIMX_HOPR_BIG", 256);
  // pass split: 0 never, 1 always, 2 (default) when the windows alone leave the CUs under-filled
  static const int64_t split_env = env_i64("AIMX_HOPR_SPLIT", 2);
  static const int64_t split_below = env_i64("AIMX_HOPR_SPLIT_BELOW", 8192);
  static const int32_t interleave = env_i64("AIMX_HOP_INTERLEAVE", 1) != 0 ? 1 : 0;
  static const bool no_seg = env_i64("AIMX_HOP_NO_SEG", 0) != 0;
  static const int64_t lds_pad = env_i64("AIMX_HOPR_LDS_PAD", 0);  // experiments: fewer workgroups per CU
  static const int32_t lean = env_i64("AIMX_HOPR_LEAN", 1) != 0 ? 1 : 0;
  static const int32_t prefetch = env_i64("AIMX_HOPR_PREFETCH", 0) != 0 ? 1 : 0;
  // column passes: the fewest equal passes of at most wc_max floats
  const int64_t passes = cdiv(D, wc_max);
  const int64_t wc = (cdiv(D, passes) + 3) / 4 * 4;
  const int64_t wu = wc / 4;
  const int64_t w_last = D - (passes - 1) * wc;
  // LDS: head + col slots + (cap rows x (wc + 4)) output tile (>= cap + 1 staged rows of wc); cap
  // rows per piece (>= the largest molecule, or it takes the global fallback), bounded by the
  // result registers
  int64_t cap = std::min<int64_t>({(int64_t)kRScan, cap_env, (int64_t)kRMaxU * kRT / wu});
  cap = std::max<int64_t>(cap, 1);
  const size_t dyn = (size_t)(kRHead + col_cap) * 4 + (size_t)(cap * (wc + 4) + wc) * 4 + lds_pad;
  const bool seg = row_seg != nullptr && !no_seg;
  const int64_t win = seg ? std::max<int64_t>(1, std::min<int64_t>(win_env, kRScan)) : cap;
  const int64_t split = (out_rpc > 0 && out_rpc < rows) ? out_rpc : rows;
  const int64_t nwin = cdiv(split, win);
  const bool pass_split = passes > 1 && (split_env == 1 || (split_env == 2 && nwin < split_below));
  const int64_t nsmall = windows ? nwin * (pass_split ? passes : 1) : 0;
  const int64_t big = std::max<int64_t>(cap, big_env);
  const int64_t nbig = cdiv(rows - split, big);
  RowsArgs a;
  a.src = src;
  a.src_ld = src_ld;
  a.src_cs = src_cs;
  a.src_rpc = make_fastdiv(src_rpc > 0 ? (uint32_t)src_rpc : 0);
  a.rowptr = rowptr;
  a.col = col;
  a.D = (uint32_t)D;
  a.wc = (uint32_t)wc;
  a.passes = (uint32_t)passes;
  a.wu_full = make_fastdiv((uint32_t)wu);
  a.wu_last = make_fastdiv((uint32_t)cdiv(w_last, 4));
  a.uo_full = make_fastdiv((uint32_t)wu + 1);
  a.uo_last = make_fastdiv((uint32_t)cdiv(w_last, 4) + 1);
  a.uo_row = make_fastdiv((uint32_t)cdiv(D, 4) + 1);
  a.rows = (uint32_t)rows;
  a.split = (uint32_t)split;
  a.win = (uint32_t)win;
  a.nwin = (uint32_t)nwin;
  a.cap = (uint32_t)cap;
  a.col_cap = (uint32_t)col_cap;
  a.pass_split = pass_split ? 1u : 0u;
  a.nsmall = (uint32_t)nsmall;
  a.big_rows = (uint32_t)big;
  a.nbig = (uint32_t)nbig;
  a.out = out;
  a.out_ld = out_ld;
  a.out_cs = out_cs;
  a.out_rpc = make_fastdiv(out_rpc > 0 ? (uint32_t)out_rpc : 0);
  a.add0 = add0;
  a.add0_ld = add0_ld;
  a.add0_early = (add0 && ((uintptr_t)add0 & 15) == 0 && add0_ld % 4 == 0) ? 1 : 0;
  a.add1 = add1;
  a.add1_ld = add1_ld;
  a.seg = seg ? row_seg : nullptr;
  a.seg_stride = row_seg_stride;
  const bool contiguous = out_ld == D && (out_rpc <= 0 || out_cs == out_rpc * out_ld);
  a.flat_zero = (contiguous && !add0 && !add1) ? 1 : 0;
  a.interleave = interleave;
  a.lean = lean;
  a.skip_tail = skip_tail;
  const int64_t blocks = nsmall + nbig;
  if (blocks <= 0) return AIMX_OK;
  if (blocks >= (int64_t)INT32_MAX) return AIMX_EARG;
  using KFn = void (*)(const RowsArgs);
  KFn fn = prefetch ? (src_rpc > 0 ? k_gather_rows<true, true> : k_gather_rows<false, true>)
                    : (src_rpc > 0 ? k_gather_rows<true, false> : k_gather_rows<false, false>);
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kRT), dyn, stream, a);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

}  // namespace aimx
