// Graph pooling kernels: multi-head attention pool and mean/max/sum, one molecule per workgroup.
//
// Reference: MultiHeadAttentionPoolingLayer.forward, src/models/pooling.py:122-172, and
// Mean/Max/SumPoolingLayer, pooling.py:15-80 (torch_scatter scatter_softmax / scatter_sum /
// scatter_mean / scatter_max). The reference materialises [H, N, hidden] (x expanded per head,
// pooling.py:150-159). Here each x row is read from HBM once per direction:
//
// * Row-resident path (every molecule up to 4·R atoms with C <= 1024, C % 4 == 0): a workgroup
//   of S·4 waves owns one molecule. Wave (s, p) holds channel slice s (256 channels, one float4 per
//   lane) of the molecule's atoms p, p+4, p+8, ... in registers, loaded in one burst. Score dot
//   products are reduced across lanes by a reduce-scatter butterfly (R·H values in ~R·H shuffles,
//   not 6·R·H) and across slices in LDS; the softmax of head h is one wave (lanes over atoms); the
//   pooled sum and, in the backward, dx and the weight-gradient partials are formed from the same
//   registers, so the backward reads x once and writes dx once.
// * General path (larger molecules, odd widths or alignment): per-molecule three-pass body that
//   re-reads x rows (L2-resident), softmax statistics in LDS or, beyond kCap atoms, global scratch.
//
// Molecules never span workgroups, so there are no atomics; weight gradients are per-molecule
// partial slabs reduced in molecule order by a second kernel (deterministic).
#include <algorithm>
#include <cstdlib>

#include "aimx_common.h"

namespace aimx {
namespace {

constexpr int kMaxH = 8;
constexpr int kCap = 512;   // atoms per molecule kept in LDS on the general path (beyond: global scratch)
constexpr int kCapB = 128;  // the same for the backward's two fp64 scratch arrays
constexpr int kSegThreads = 256;
constexpr int kGeneralSmem = 16 * 1024;
static_assert(kMaxH * kCap * 4 <= kGeneralSmem && 2 * kMaxH * kCapB * 8 <= kGeneralSmem, "general-path scratch fits");

template <int NW>
__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += red[i];
  return s;
}

template <int NW>
__device__ __forceinline__ float block_reduce_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) s = fmaxf(s, red[i]);
  return s;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int NW>
__device__ __forceinline__ double block_reduce_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += red[i];
  return s;
}

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }
constexpr int pow2ceil(int v) { return v <= 1 ? 1 : 2 * pow2ceil((v + 1) / 2); }

// Sum NV per-lane values over the wave's 64 lanes. Each butterfly step sends half of the values a
// lane still holds to its partner and keeps the other half, so the whole reduction costs
// NV - 1 + log2(64 / NV) shuffles instead of 6·NV. On return each lane holds the wave total of
// value index lane >> (6 - log2 NV) (lanes of one group of 64 / NV hold the same total).
// (Template recursion keeps every step's trip count a constant, so v stays in registers.)
template <int M, int O, typename T>
struct RsStep {
  static __device__ __forceinline__ void run(T* v, int lane) {
    const bool up = (lane & O) != 0;
#pragma unroll
    for (int i = 0; i < M / 2; ++i) {
      const T send = up ? v[i] : v[i + M / 2];
      const T keep = up ? v[i + M / 2] : v[i];
      v[i] = keep + __shfl_xor(send, O, 64);
    }
    RsStep<M / 2, O / 2, T>::run(v, lane);
  }
};
template <int O, typename T>
struct RsStep<1, O, T> {
  static __device__ __forceinline__ void run(T*, int) {}
};

template <int NV, typename T>
__device__ __forceinline__ T wave_reduce_scatter(T (&v)[NV]) {
  static_assert(NV >= 1 && NV <= 64 && (NV & (NV - 1)) == 0, "NV: power of two <= 64");
  const int lane = threadIdx.x & 63;
  RsStep<NV, 32, T>::run(v, lane);
  T r = v[0];
#pragma unroll
  for (int o = 32 >> ilog2(NV); o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
  return r;
}

// Per-(head, atom) scratch for one molecule: LDS image [H][kCap] when the molecule fits, else the
// global [H][N] arrays. Two inlined instantiations keep every access in one address space.
template <bool LDS, typename T = float, int CAP = kCap>
struct Slot {
  T* p;
  int64_t N;
  __device__ __forceinline__ T& at(int h, int j, int64_t i) const { return LDS ? p[h * CAP + j] : p[h * N + i]; }
};

// ---------------------------------------------------------------------------------------------
// General path (any molecule size, width or alignment)
// ---------------------------------------------------------------------------------------------
template <bool LDS, int NT>
__device__ __forceinline__ void attn_fwd_body(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, const float* __restrict__ bias, float tau,
                                              int H, int32_t b, int n, const int32_t* __restrict__ gperm, int g,
                                              float* __restrict__ pooled, float* __restrict__ attn,
                                              float* __restrict__ scores, Slot<LDS> sa, float* red) {
  constexpr int NW = NT / kWave;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // 1) scores, centred on the first atom (fp64 dots; the softmax is shift invariant and the bias
  //    cancels: d_hj = (x_j - x_0) . W_h / tau, see attn_fwd_rows), a wave per atom, lanes over
  //    channels; d is kept in LDS or, for the largest molecules, in the scores array itself
  const int64_t i0 = n > 0 ? gperm[b] : 0;  // (an empty molecule reads no row)
  for (int j = w; j < n; j += NW) {
    const int64_t i = gperm[b + j];
    double acc[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) acc[h] = 0.0;
    for (int64_t c = lane; c < C; c += 64) {
      const double xv = (double)x[i * ldx + c] - (double)x[i0 * ldx + c];
#pragma unroll
      for (int h = 0; h < kMaxH; ++h)
        if (h < H) acc[h] += xv * (double)W[h * C + c];
    }
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) {
      if (h < H) {
        const float d = (float)(wave_sum_d(acc[h]) / (double)tau);
        if (lane == 0) {
          if (LDS)
            sa.at(h, j, i) = d;
          else
            scores[h * N + i] = d;
        }
      }
    }
  }
  if (!LDS) __threadfence();
  __syncthreads();
  // 2) per-head softmax over the molecule's atoms (torch_scatter.scatter_softmax); the saved
  //    scores are s_0 + d with s_0 = (x_0 . W_h + b_h) / tau
  for (int h = 0; h < H; ++h) {
    double s0 = 0.0;
    for (int64_t c = lane; c < C; c += 64) s0 += (double)x[i0 * ldx + c] * (double)W[h * C + c];
    s0 = (wave_sum_d(s0) + (double)bias[h]) / (double)tau;
    float mx = -INFINITY;
    for (int j = threadIdx.x; j < n; j += NT) mx = fmaxf(mx, LDS ? sa.at(h, j, 0) : scores[h * N + gperm[b + j]]);
    mx = block_reduce_max<NW>(mx, red);
    float sum = 0.f;
    for (int j = threadIdx.x; j < n; j += NT) sum += expf((LDS ? sa.at(h, j, 0) : scores[h * N + gperm[b + j]]) - mx);
    sum = block_reduce_sum<NW>(sum, red);
    for (int j = threadIdx.x; j < n; j += NT) {
      const int64_t i = gperm[b + j];
      const float d = LDS ? sa.at(h, j, i) : scores[h * N + i];
      const float a = expf(d - mx) / sum;
      attn[h * N + i] = a;
      scores[h * N + i] = (float)(s0 + (double)d);
      if (LDS) sa.at(h, j, i) = a;
    }
    if (!LDS) __threadfence();
    __syncthreads();  // this head's d values are consumed before the next head's reads start
  }
  // 3) pooled[g,c] = (sum_h sum_i a[h,i] x[i,c]) / H  (pooling.py:150-161: per-head sums, head mean)
  for (int64_t c = threadIdx.x; c < C; c += NT) {
    float acc[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) acc[h] = 0.f;
    for (int j = 0; j < n; ++j) {
      const int64_t i = gperm[b + j];
      const float xv = x[i * ldx + c];
#pragma unroll
      for (int h = 0; h < kMaxH; ++h)
        if (h < H) acc[h] += (LDS ? sa.at(h, j, i) : attn[h * N + i]) * xv;
    }
    float s = 0.f;
#pragma unroll
    for (int h = 0; h < kMaxH; ++h)
      if (h < H) s += acc[h];
    pooled[(int64_t)g * C + c] = s / (float)H;
  }
}

// Backward. ds[h,i] = a (da - sum_j a da), da[h,i] = (x_i . dpooled[g]) / H + d_attn[h,i].
// The softmax backward cancels (da - <a, da>) when a molecule's attention is peaked, so every
// reduction here (dots, <a, da>, ds, the dW/db/dtau partial sums) is accumulated in fp64: the
// kernel is memory/latency-bound and the fp64 VALU rate is not the limit.
template <bool LDS, int NT>
__device__ __forceinline__ void attn_bwd_body(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, float tau, int H, int32_t b, int n,
                                              const int32_t* __restrict__ gperm, int g,
                                              const float* __restrict__ attn, const float* __restrict__ scores,
                                              const float* __restrict__ dpool, const float* __restrict__ dattn,
                                              float* __restrict__ dx, int64_t lddx, float* __restrict__ dW_part,
                                              double* __restrict__ db_part, double* __restrict__ dtau_part,
                                              Slot<LDS, double, kCapB> sds, Slot<LDS, double, kCapB> sxw,
                                              double* red) {
  constexpr int NW = NT / kWave;
  const double invH = 1.0 / (double)H;
  const double dtau_inv = 1.0 / (double)tau;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* q = dpool + (int64_t)g * C;
  // 1) da[h,i], and x_i . W_h in fp64 for the temperature gradient (see attn_bwd_rows)
  for (int j = w; j < n; j += NW) {
    const int64_t i = gperm[b + j];
    double acc = 0.0, aw[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) aw[h] = 0.0;
    for (int64_t c = lane; c < C; c += 64) {
      const double xv = x[i * ldx + c];
      acc += xv * (double)q[c];
#pragma unroll
      for (int h = 0; h < kMaxH; ++h)
        if (h < H) aw[h] += xv * (double)W[h * C + c];
    }
    const double d = wave_sum_d(acc) * invH;
    if (lane < H) sds.at(lane, j, i) = d + (dattn ? (double)dattn[lane * N + i] : 0.0);
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) {
      if (h < H) {
        const double sw = wave_sum_d(aw[h]);
        if (lane == 0) sxw.at(h, j, i) = sw;
      }
    }
  }
  if (!LDS) __threadfence();
  __syncthreads();
  // 2) ds = a (da - <a, da>) per head; db and dtau partials
  double dtau_acc = 0.0;
  for (int h = 0; h < H; ++h) {
    // t = <a, da> / sum(a): normalising by the fp32 weights' actual sum keeps sum_i ds = 0 exactly
    // (the softmax is shift invariant). Without it the (1 - sum a) rounding residue times t leaks
    // a common-mode term into every ds, which dW = sum ds x amplifies wherever the atoms' features
    // share a large mean. (torch's autograd gets the same cancellation by routing the residue
    // through scatter_max's gradient.)
    double t = 0.0, asum = 0.0;
    for (int j = threadIdx.x; j < n; j += NT) {
      const int64_t i = gperm[b + j];
      const double a = attn[h * N + i];
      t += a * sds.at(h, j, i);
      asum += a;
    }
    t = block_reduce_sum_d<NW>(t, red);
    asum = block_reduce_sum_d<NW>(asum, red);
    if (asum > 0.0) t /= asum;
    double dbs = 0.0;
    for (int j = threadIdx.x; j < n; j += NT) {
      const int64_t i = gperm[b + j];
      const double ds = (double)attn[h * N + i] * (sds.at(h, j, i) - t);
      sds.at(h, j, i) = ds;
      dbs += ds;
      dtau_acc += ds * sxw.at(h, j, i) * dtau_inv;  // s without the bias: sum_i ds = 0
    }
    dbs = block_reduce_sum_d<NW>(dbs, red);
    if (threadIdx.x == 0) db_part[(int64_t)g * H + h] = dbs * dtau_inv;
  }
  dtau_acc = block_reduce_sum_d<NW>(dtau_acc, red);
  if (threadIdx.x == 0) dtau_part[g] = -dtau_acc * dtau_inv;
  if (!LDS) __threadfence();
  __syncthreads();
  // 3) dx_i = (sum_h a[h,i]) q / H + sum_h ds[h,i] W_h / tau ; dW_part[g,h] = sum_i ds[h,i] x_i / tau
  for (int64_t c = threadIdx.x; c < C; c += NT) {
    const double qc = (double)q[c] * invH;
    double wc[kMaxH], dw[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) {
      wc[h] = h < H ? (double)W[h * C + c] : 0.0;
      dw[h] = 0.0;
    }
    for (int j = 0; j < n; ++j) {
      const int64_t i = gperm[b + j];
      const double xv = x[i * ldx + c];
      double asum = 0.0, dsw = 0.0;
#pragma unroll
      for (int h = 0; h < kMaxH; ++h) {
        if (h < H) {
          const double ds = sds.at(h, j, i);
          asum += attn[h * N + i];
          dsw += ds * wc[h];
          dw[h] += ds * xv;
        }
      }
      dx[i * lddx + c] = (float)(asum * qc + dsw * dtau_inv);
    }
#pragma unroll
    for (int h = 0; h < kMaxH; ++h)
      if (h < H) dW_part[((int64_t)g * H + h) * C + c] = (float)(dw[h] * dtau_inv);
  }
}

// ---------------------------------------------------------------------------------------------
// Row-resident path
// ---------------------------------------------------------------------------------------------
constexpr int kMaxAtomsRows = 128;  // molecules up to this many atoms take the row-resident path

__device__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

__device__ __forceinline__ float4 sub4(float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }

__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

__device__ __forceinline__ float4 scale4(float4 a, float k) { return make_float4(a.x * k, a.y * k, a.z * k, a.w * k); }

// k * a + c, per component
__device__ __forceinline__ float4 fma4(float k, float4 a, float4 c) {
  return make_float4(fmaf(k, a.x, c.x), fmaf(k, a.y, c.y), fmaf(k, a.z, c.z), fmaf(k, a.w, c.w));
}

__device__ __forceinline__ double dot4d(float4 a, float4 b) {
  return (double)a.x * (double)b.x + (double)a.y * (double)b.y + (double)a.z * (double)b.z + (double)a.w * (double)b.w;
}

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// The row-resident paths read x through a raw buffer descriptor (aimx_common.h buffer_rsrc): its
// extent ends at the last row's C-th channel, so the 32-bit byte offsets need (N-1)·ldx + C < 2^30.
__device__ __forceinline__ bool rows_addressable(int64_t N, int64_t ldx, int64_t C) {
  return (N - 1) * ldx + C < ((int64_t)1 << 30) - 4;
}
__device__ __forceinline__ uint32_t rows_extent(int64_t N, int64_t ldx, int64_t C) {
  return 4u * (uint32_t)max<int64_t>((N - 1) * ldx + C, 1);
}

typedef float pfloatx4 __attribute__((ext_vector_type(4)));

// This wave's rows j = base + p + r*P of the molecule (n >= 1 atoms), lane channels c..c+3, in two
// rounds: the R row indices (clamped into the molecule, so always valid loads), then the R rows; an
// invalid row or channel is an ADDRESS select past the extent (reads 0). A value select per row
// (`valid ? load : 0`) makes hipcc branch around each load and wait for it: R dependent round trips
// instead of two. (Round 4 reverted this form after a fault; the cause was the descriptor's
// sign-extended base, see buffer_rsrc, not these offsets.)
template <int P, int R>
__device__ __forceinline__ void load_rows(float4 (&xr)[R], __amdgpu_buffer_rsrc_t rx, uint32_t xbytes, int64_t ldx,
                                          const int32_t* __restrict__ gperm, int32_t b, int n, int base, int p,
                                          int c, bool cv) {
  int32_t q[R];
#pragma unroll
  for (int r = 0; r < R; ++r) q[r] = gperm[b + max(min(base + p + r * P, n - 1), 0)];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = base + p + r * P;
    const uint32_t off = (cv && j < n) ? 4u * (uint32_t)((int64_t)q[r] * ldx + c) : xbytes;
    const pfloatx4 v = __builtin_bit_cast(pfloatx4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
    xr[r] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Forward. A molecule of up to P·R atoms is one chunk and stays in registers from the score pass
// to the pooled sum; larger ones (up to kMaxAtomsRows) run chunk by chunk and reload each chunk
// for the pooled sum (L2/MALL hits).
//
// Centering. The softmax is shift invariant, so the scores enter as d_hj = (x_j - x_0) . W_h / tau
// (x_0 = the molecule's first row; the bias cancels): fp32 dots of centred rows keep their error
// relative to the spread of the scores, not to their common level (plain fp32 score sums left
// 1e-6..6e-5 of the temperature gradient, which cancels the same way, to the summation order).
// The saved scores are s_0 + d with s_0 = (x_0 . W_h + b_h) / tau.
//
// LDS (floats): scp [S][HM][MAXA] per-slice partial dots (+ [S][HM] of x_0 . W_h), sa [HM][MAXA]
// attention, red [P-1][S*256] pooled partials.
template <int S, int P, int R, int HM>
__device__ __forceinline__ void attn_fwd_rows(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, const float* __restrict__ bias, float tau,
                                              int H, int32_t b, int n, const int32_t* __restrict__ gperm, int g,
                                              float* __restrict__ pooled, float* __restrict__ attn,
                                              float* __restrict__ scores, char* smem) {
  constexpr int CAPN = P * R, NW = S * P, SC = S * 256, MAXA = kMaxAtomsRows;
  // (R + 1) x HM dot partials (the extra row: x_0 . W_h) reduced in groups of NVC (power of two
  // <= 32, the last group zero-padded)
  constexpr int NV = (R + 1) * HM, NVC = NV >= 32 ? 32 : pow2ceil(NV), NCH = (NV + NVC - 1) / NVC,
                SH = 6 - ilog2(NVC);
  float* scp = reinterpret_cast<float*>(smem);
  float* s0p = scp + S * HM * MAXA;
  float* sa = s0p + S * HM;
  float* red = sa + HM * MAXA;
  // wave index made scalar: row indices, gperm reads and LDS offsets below stay in SGPRs
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), s = w % S, p = w / S;
  const int c = s * 256 + lane * 4;
  const bool cv = c < C;
  const int nchunk = (n + CAPN - 1) / CAPN;
  const uint32_t xbytes = rows_extent(N, ldx, C);
  const __amdgpu_buffer_rsrc_t rx = buffer_rsrc(x, xbytes);
  const float4 x0 = (cv && n > 0) ? ld4(x + (int64_t)gperm[b] * ldx + c) : zero4();
  float4 wv[HM];
#pragma unroll
  for (int h = 0; h < HM; ++h) wv[h] = (cv && h < H) ? ld4(W + (int64_t)h * C + c) : zero4();
  float4 xr[R];
  // 1) partial dots of this slice, reduced across the wave
  for (int ch = 0; ch < nchunk; ++ch) {
    const int base = ch * CAPN;
    load_rows<P, R>(xr, rx, xbytes, ldx, gperm, b, n, base, p, c, cv);
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      float v[NVC];
#pragma unroll
      for (int k = 0; k < NVC; ++k) {
        const int idx = q * NVC + k, r = idx / HM;
        v[k] = idx >= NV ? 0.f : (r < R ? dot4(sub4(xr[r], x0), wv[idx % HM]) : dot4(x0, wv[idx % HM]));
      }
      const float tot = wave_reduce_scatter<NVC>(v);
      const int idx = q * NVC + (lane >> SH);
      const int r = idx / HM, h = idx % HM, j = base + p + r * P;
      if ((lane & ((1 << SH) - 1)) == 0 && idx < NV && h < H) {
        if (r < R) {
          if (j < n) scp[(s * HM + h) * MAXA + j] = tot;
        } else if (ch == 0 && p == 0) {
          s0p[s * HM + h] = tot;
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one group's products live at a time (VGPR budget)
    }
  }
  __syncthreads();
  // 2) softmax of head h by one wave, lanes over atoms
  const float inv_tau = 1.f / tau;
  for (int h = w; h < H; h += NW) {
    float s0 = 0.f;
#pragma unroll
    for (int k = 0; k < S; ++k) s0 += s0p[k * HM + h];
    s0 = (s0 + bias[h]) * inv_tau;
    float mx = -INFINITY;
    for (int j = lane; j < n; j += 64) {
      float d = 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) d += scp[(k * HM + h) * MAXA + j];
      d *= inv_tau;
      sa[h * MAXA + j] = d;
      mx = fmaxf(mx, d);
    }
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < n; j += 64) sum += expf(sa[h * MAXA + j] - mx);
    sum = wave_sum(sum);
    for (int j = lane; j < n; j += 64) {
      const int64_t i = gperm[b + j];
      const float d = sa[h * MAXA + j];
      const float a = expf(d - mx) / sum;
      scores[h * N + i] = s0 + d;
      attn[h * N + i] = a;
      sa[h * MAXA + j] = a;
    }
  }
  __syncthreads();
  // 3) pooled[g] = (1/H) sum_i (sum_h a[h,i]) x_i : this wave's rows, then the row groups in order
  float4 acc = zero4();
  for (int ch = 0; ch < nchunk; ++ch) {
    const int base = ch * CAPN;
    if (nchunk > 1) load_rows<P, R>(xr, rx, xbytes, ldx, gperm, b, n, base, p, c, cv);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = base + p + r * P;
      if (j < n) {
        float cf = 0.f;
#pragma unroll
        for (int h = 0; h < HM; ++h)
          if (h < H) cf += sa[h * MAXA + j];
        acc = fma4(cf, xr[r], acc);
      }
    }
  }
  if (p > 0 && cv) *reinterpret_cast<float4*>(red + (p - 1) * SC + c) = acc;
  __syncthreads();
  if (p == 0 && cv) {
#pragma unroll
    for (int k = 0; k < P - 1; ++k) acc = add4(acc, *reinterpret_cast<const float4*>(red + k * SC + c));
    const float invH = 1.f / (float)H;
    *reinterpret_cast<float4*>(pooled + (int64_t)g * C + c) =
        make_float4(acc.x * invH, acc.y * invH, acc.z * invH, acc.w * invH);
  }
}

// Backward (same chunking and centring: x_j - x_0 in every dot; sum_j ds_hj = 0, so the
// centred da, score and dW sums equal the plain ones exactly, and fp32 keeps their error relative
// to the spread of the atoms' features rather than their common level).
//   da_hj = (x_j - x_0) . q / H + d_attn_hj,  t_h = sum_j a da / sum_j a,  ds = a (da - t)
//   dx_j = (sum_h a_hj) q / H + sum_h ds_hj W_h / tau
//   dW_h = sum_j ds_hj (x_j - x_0) / tau,  db_h = sum_j ds_hj / tau,
//   dtau = -sum_hj ds_hj ((x_j - x_0) . W_h / tau) / tau
// LDS (floats): dap [S][MAXA] per-slice x.q partials, dsp [S][HM][MAXA] x.W_h partials, sds [HM][MAXA]
// ds, sa [HM][MAXA] attention, red [P-1][HM][S*256] dW partials; dtp [NW] doubles.
template <int S, int P, int R, int HM>
__device__ __forceinline__ void attn_bwd_rows(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, float tau, int H, int32_t b, int n,
                                              const int32_t* __restrict__ gperm, int g,
                                              const float* __restrict__ attn, const float* __restrict__ dpool,
                                              const float* __restrict__ dattn, float* __restrict__ dx, int64_t lddx,
                                              float* __restrict__ dW_part, double* __restrict__ db_part,
                                              double* __restrict__ dtau_part, char* smem) {
  constexpr int CAPN = P * R, NW = S * P, SC = S * 256, MAXA = kMaxAtomsRows;
  // per row: x.q and the HM x.W_h dots, reduced in groups of NVC (power of two <= 32, zero-padded)
  constexpr int HC = HM + 1, NV = R * HC, NVC = NV >= 32 ? 32 : pow2ceil(NV), NCH = (NV + NVC - 1) / NVC,
                SH = 6 - ilog2(NVC);
  double* dtp = reinterpret_cast<double*>(smem);
  float* dap = reinterpret_cast<float*>(dtp + NW);
  float* dsp = dap + S * MAXA;
  float* sds = dsp + S * HM * MAXA;
  float* sa = sds + HM * MAXA;
  float* red = sa + HM * MAXA;
  // wave index made scalar: row indices, gperm reads and LDS offsets below stay in SGPRs
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), s = w % S, p = w / S;
  const int c = s * 256 + lane * 4;
  const bool cv = c < C;
  const int nchunk = (n + CAPN - 1) / CAPN;
  const uint32_t xbytes = rows_extent(N, ldx, C);
  const __amdgpu_buffer_rsrc_t rx = buffer_rsrc(x, xbytes);
  const float4 x0 = (cv && n > 0) ? ld4(x + (int64_t)gperm[b] * ldx + c) : zero4();
  const float4 q = cv ? ld4(dpool + (int64_t)g * C + c) : zero4();
  float4 wv[HM];
#pragma unroll
  for (int h = 0; h < HM; ++h) wv[h] = (cv && h < H) ? ld4(W + (int64_t)h * C + c) : zero4();
  for (int t = threadIdx.x; t < H * n; t += NW * 64) {
    const int h = t / n, j = t - h * n;
    sa[h * MAXA + j] = attn[h * N + gperm[b + j]];
  }
  float4 xr[R];
  // 1) centred dots with q and with each W_h for this slice, reduced across the wave
  for (int ch = 0; ch < nchunk; ++ch) {
    const int base = ch * CAPN;
    load_rows<P, R>(xr, rx, xbytes, ldx, gperm, b, n, base, p, c, cv);
#pragma unroll
    for (int qq = 0; qq < NCH; ++qq) {
      float v[NVC];
#pragma unroll
      for (int k = 0; k < NVC; ++k) {
        const int idx = qq * NVC + k;
        v[k] = idx < NV ? dot4(sub4(xr[idx / HC], x0), (idx % HC) == 0 ? q : wv[(idx % HC + HM - 1) % HM]) : 0.f;
      }
      const float tot = wave_reduce_scatter<NVC>(v);
      const int idx = qq * NVC + (lane >> SH);
      const int r = idx / HC, comp = idx % HC, j = base + p + r * P;
      if ((lane & ((1 << SH) - 1)) == 0 && idx < NV && j < n) {
        if (comp == 0)
          dap[s * MAXA + j] = tot;
        else if (comp - 1 < H)
          dsp[(s * HM + comp - 1) * MAXA + j] = tot;
      }
      __builtin_amdgcn_sched_barrier(0);  // one group's products live at a time (VGPR budget)
    }
  }
  __syncthreads();
  // 2) ds = a (da - <a, da> / sum a) per head (one wave per head, lanes over atoms; sums in fp64);
  //    db, dtau partials (normalising by sum a keeps sum_i ds = 0: see attn_bwd_body)
  const double invH = 1.0 / (double)H;
  const double dtau_inv = 1.0 / (double)tau;
  double dtl = 0.0;
  for (int h = w; h < H; h += NW) {
    double t = 0.0, asum = 0.0;
    for (int j = lane; j < n; j += 64) {
      float d = 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) d += dap[k * MAXA + j];
      const double da = (double)d * invH + (dattn ? (double)dattn[h * N + gperm[b + j]] : 0.0);
      const double a = sa[h * MAXA + j];
      sds[h * MAXA + j] = (float)da;  // exact up to its fp32 rounding: recomputed below
      t += a * da;
      asum += a;
    }
    t = wave_sum_d(t);
    asum = wave_sum_d(asum);
    if (asum > 0.0) t /= asum;
    double dbs = 0.0;
    for (int j = lane; j < n; j += 64) {
      float d = 0.f, sw = 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        d += dap[k * MAXA + j];
        sw += dsp[(k * HM + h) * MAXA + j];
      }
      const double da = (double)d * invH + (dattn ? (double)dattn[h * N + gperm[b + j]] : 0.0);
      const double ds = (double)sa[h * MAXA + j] * (da - t);
      sds[h * MAXA + j] = (float)ds;
      dbs += ds;
      dtl += ds * (double)sw * dtau_inv;
    }
    dbs = wave_sum_d(dbs);
    if (lane == 0) db_part[(int64_t)g * H + h] = dbs * dtau_inv;
  }
  dtl = wave_sum_d(dtl);
  if (lane == 0) dtp[w] = dtl;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < NW; ++k) t += dtp[k];
    dtau_part[g] = -t * dtau_inv;
  }
  // 3) dx_j = (sum_h a_hj) q / H + sum_h ds_hj W_h / tau, and dW partials sum_j ds_hj (x_j - x_0)
  const float qh = 1.f / (float)H, ti = 1.f / tau;
  const float4 qs = make_float4(q.x * qh, q.y * qh, q.z * qh, q.w * qh);
  float4 dw[HM];
#pragma unroll
  for (int h = 0; h < HM; ++h) dw[h] = zero4();
  for (int ch = 0; ch < nchunk; ++ch) {
    const int base = ch * CAPN;
    if (nchunk > 1) load_rows<P, R>(xr, rx, xbytes, ldx, gperm, b, n, base, p, c, cv);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = base + p + r * P;
      if (j < n) {
        const float4 xc = sub4(xr[r], x0);
        float as = 0.f;
        float4 d = zero4();
#pragma unroll
        for (int h = 0; h < HM; ++h) {
          if (h < H) {
            const float ds = sds[h * MAXA + j];
            as += sa[h * MAXA + j];
            d = fma4(ds, wv[h], d);
            dw[h] = fma4(ds, xc, dw[h]);
          }
        }
        if (cv) *reinterpret_cast<float4*>(dx + (int64_t)gperm[b + j] * lddx + c) = fma4(as, qs, scale4(d, ti));
      }
    }
  }
  // 4) this molecule's dW partial: the row groups combined in order, all heads at once
  if (p > 0 && cv) {
#pragma unroll
    for (int h = 0; h < HM; ++h)
      if (h < H) *reinterpret_cast<float4*>(red + ((p - 1) * HM + h) * SC + c) = dw[h];
  }
  __syncthreads();
  if (p == 0 && cv) {
#pragma unroll
    for (int h = 0; h < HM; ++h) {
      if (h < H) {
        float4 t = dw[h];
#pragma unroll
        for (int k = 0; k < P - 1; ++k) t = add4(t, *reinterpret_cast<const float4*>(red + (k * HM + h) * SC + c));
        *reinterpret_cast<float4*>(dW_part + ((int64_t)g * H + h) * C + c) = scale4(t, ti);
      }
    }
  }
}

template <int S, int P, int HM>
constexpr int rows_fwd_bytes() {
  return 4 * (S * HM * kMaxAtomsRows + S * HM + HM * kMaxAtomsRows + (P - 1) * S * 256);
}
template <int S, int P, int HM>
constexpr int rows_bwd_bytes() {
  return 8 * S * P + 4 * (S * kMaxAtomsRows + S * HM * kMaxAtomsRows + 2 * HM * kMaxAtomsRows + (P - 1) * HM * S * 256);
}
template <int S, int P, int HM>
constexpr int smem_bytes() {
  return std::max(kGeneralSmem, std::max(rows_fwd_bytes<S, P, HM>(), rows_bwd_bytes<S, P, HM>()));
}

// One molecule per workgroup of S*P waves. The row-resident body runs when the molecule and the
// operand layout fit it (a per-block uniform choice); the general body otherwise.
template <int S, int P, int R, int HM>
__global__ __launch_bounds__(S * P * 64) void k_attn_fwd(
    const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ tau_p, int H, const int32_t* __restrict__ gptr,
    const int32_t* __restrict__ gperm, float* __restrict__ pooled, float* __restrict__ attn,
    float* __restrict__ scores) {
  constexpr int NT = S * P * 64;
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<S, P, HM>()];
  __shared__ float red[NT / 64];
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  const int n = e - b;
  const float tau = *tau_p;
  const bool rows = n <= kMaxAtomsRows && H <= HM && C <= S * 256 && (C % 4) == 0 &&
                    (ldx % 4) == 0 && al16(x) && al16(W) && al16(pooled) && rows_addressable(N, ldx, C);
  if (rows)
    attn_fwd_rows<S, P, R, HM>(x, ldx, N, C, W, bias, tau, H, b, n, gperm, g, pooled, attn, scores, smem);
  else if (n <= kCap)
    attn_fwd_body<true, NT>(x, ldx, N, C, W, bias, tau, H, b, n, gperm, g, pooled, attn, scores,
                            Slot<true>{reinterpret_cast<float*>(smem), N}, red);
  else
    attn_fwd_body<false, NT>(x, ldx, N, C, W, bias, tau, H, b, n, gperm, g, pooled, attn, scores, Slot<false>{attn, N},
                             red);
}

template <int S, int P, int R, int HM>
__global__ __launch_bounds__(S * P * 64) void k_attn_bwd(
    const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C, const float* __restrict__ W,
    const float* __restrict__ tau_p, int H, const int32_t* __restrict__ gptr, const int32_t* __restrict__ gperm,
    const float* __restrict__ attn, const float* __restrict__ scores, const float* __restrict__ dpool,
    const float* __restrict__ dattn, float* __restrict__ dx, int64_t lddx, float* __restrict__ dW_part,
    double* __restrict__ db_part, double* __restrict__ dtau_part, double* __restrict__ ds_glob,
    int32_t* __restrict__ red_cnt, int n_red_cnt) {
  constexpr int NT = S * P * 64;
  // the arrival counters of the fused partial reduction (k_attn_reduce) that follows this launch
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < n_red_cnt; i += NT) red_cnt[i] = 0;
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<S, P, HM>()];
  __shared__ double red[NT / 64];
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  const int n = e - b;
  const float tau = *tau_p;
  const bool rows = n <= kMaxAtomsRows && H <= HM && C <= S * 256 && (C % 4) == 0 &&
                    (ldx % 4) == 0 && (lddx % 4) == 0 && al16(x) && al16(W) && al16(dx) && al16(dpool) &&
                    al16(dW_part) && rows_addressable(N, ldx, C);
  if (rows)
    attn_bwd_rows<S, P, R, HM>(x, ldx, N, C, W, tau, H, b, n, gperm, g, attn, dpool, dattn, dx, lddx, dW_part, db_part,
                            dtau_part, smem);
  else if (n <= kCapB)
    attn_bwd_body<true, NT>(x, ldx, N, C, W, tau, H, b, n, gperm, g, attn, scores, dpool, dattn, dx, lddx, dW_part,
                            db_part, dtau_part, Slot<true, double, kCapB>{reinterpret_cast<double*>(smem), N},
                            Slot<true, double, kCapB>{reinterpret_cast<double*>(smem) + kMaxH * kCapB, N}, red);
  else
    attn_bwd_body<false, NT>(x, ldx, N, C, W, tau, H, b, n, gperm, g, attn, scores, dpool, dattn, dx, lddx, dW_part,
                             db_part, dtau_part, Slot<false, double, kCapB>{ds_glob, N},
                             Slot<false, double, kCapB>{ds_glob + (int64_t)H * N, N}, red);
}

// Deterministic reduction of the per-molecule partials, column t of [dW (H*C) | db (H) | dtau],
// in two launches so that enough CUs share the reads (one 64-column block per CU was bound by the
// CU's outstanding-request limit at ~10 GB/s): k_attn_reduce1 sums slices of kRedSlice molecules
// (a 64-column x 64-molecule tile per workgroup: 4 waves x 16 molecules, 16 loads in flight per
// lane, then the 4 wave sums in order) into a slice slab; k_attn_reduce2 sums the slices in order.
constexpr int kRedSlice = 64;

// Column t of [dW (H*C) | db (H) | dtau] summed over molecules g0 .. g0 + kRedSlice / 4 - 1 (those < G),
// in that order. Every load
// of the column is issued unconditionally (the molecule index clamped, out-of-range terms zeroed
// after an empty asm holds the loads), so the 16 loads per lane are in flight together; a guarded
// load per term made the compiler wait for each one at its branch's join.
__device__ __forceinline__ void hold_d(const double& v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ double slice_sum(int64_t t, int64_t g0, int64_t G, int64_t nw, int H,
                                            const float* __restrict__ dW_part, const double* __restrict__ db_part,
                                            const double* __restrict__ dtau_part) {
  constexpr int K = kRedSlice / 4;
  double v[K];
  if (t < nw) {
    float f[K];
#pragma unroll
    for (int k = 0; k < K; ++k) f[k] = dW_part[min(g0 + k, G - 1) * nw + t];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = (double)f[k];
  } else {
    const double* p = t < nw + H ? db_part + (t - nw) : dtau_part;
    const int64_t st = t < nw + H ? H : 1;
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = p[min(g0 + k, G - 1) * st];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) hold_d(v[k]);
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) s += g0 + k < G ? v[k] : 0.0;
  return s;
}

__global__ __launch_bounds__(256) void k_attn_reduce1(int64_t G, int H, int64_t C, const float* __restrict__ dW_part,
                                                      const double* __restrict__ db_part,
                                                      const double* __restrict__ dtau_part, double* __restrict__ slab) {
  __shared__ double red[4][64];
  const int64_t nw = (int64_t)H * C, tot = nw + H + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  const int64_t g0 = (int64_t)blockIdx.y * kRedSlice + w * (kRedSlice / 4);
  double s = 0.0;
  if (t < tot && g0 < G) s = slice_sum(t, g0, G, nw, H, dW_part, db_part, dtau_part);
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && t < tot) slab[(int64_t)blockIdx.y * tot + t] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

__global__ __launch_bounds__(256) void k_attn_reduce2(int64_t n_slices, int H, int64_t C, const double* __restrict__ slab,
                                                      float* __restrict__ dW, float* __restrict__ db,
                                                      float* __restrict__ dtau) {
  const int64_t nw = (int64_t)H * C, tot = nw + H + 1;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= tot) return;
  double s = 0.0;
  for (int64_t k = 0; k < n_slices; ++k) s += slab[k * tot + t];
  if (t < nw)
    dW[t] = (float)s;
  else if (t < nw + H)
    db[t - nw] = (float)s;
  else
    *dtau = (float)s;
}

// Both levels in one launch: the k_attn_reduce1 tile, its slice slab stored device-coherent, and
// the last-arriving workgroup of each 64-column block sums the block's slices in slice order (the
// same order and fp64 sums as k_attn_reduce2: bit-identical results). Hand-off as the split-K GEMM
// slabs (MI355X_MICROARCH.md "Valid forms" row 1): agent-scope slab stores, every storing wave
// drained before the workgroup barrier, one agent-scope arrival add, agent-scope slab loads. The
// counters are zeroed by the k_attn_bwd launch that precedes this one on the stream.
__global__ __launch_bounds__(256) void k_attn_reduce(int64_t G, int H, int64_t C, const float* __restrict__ dW_part,
                                                     const double* __restrict__ db_part,
                                                     const double* __restrict__ dtau_part, double* __restrict__ slab,
                                                     int32_t* __restrict__ cnt, float* __restrict__ dW,
                                                     float* __restrict__ db, float* __restrict__ dtau) {
  __shared__ double red[4][64];
  __shared__ int last;
  const int64_t nw = (int64_t)H * C, tot = nw + H + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  const int64_t g0 = (int64_t)blockIdx.y * kRedSlice + w * (kRedSlice / 4);
  double s = 0.0;
  if (t < tot && g0 < G) s = slice_sum(t, g0, G, nw, H, dW_part, db_part, dtau_part);
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && t < tot) {
    const double r = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(slab + (int64_t)blockIdx.y * tot + t),
                       __builtin_bit_cast(unsigned long long, r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(cnt + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (int)gridDim.y - 1;
  __syncthreads();
  if (!last || w != 0 || t >= tot) return;
  const int64_t ns = gridDim.y;
  double acc = 0.0;
  for (int64_t k0 = 0; k0 < ns; k0 += 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      v[k] = k0 + k < ns ? __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<unsigned long long*>(
                                                                           slab + (k0 + k) * tot + t),
                                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                         : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k0 + k < ns) acc += v[k];
  }
  if (t < nw)
    dW[t] = (float)acc;
  else if (t < nw + H)
    db[t - nw] = (float)acc;
  else
    *dtau = (float)acc;
}

// kind: 0 mean, 1 max, 2 sum
__global__ __launch_bounds__(kSegThreads) void k_segpool_fwd(int kind, const float* __restrict__ x, int64_t ldx,
                                                              int64_t C, const int32_t* __restrict__ gptr,
                                                              const int32_t* __restrict__ gperm,
                                                              float* __restrict__ out, int32_t* __restrict__ argmax) {
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  for (int64_t c = threadIdx.x; c < C; c += kSegThreads) {
    if (kind == 1) {
      // torch_scatter 2.1.2 CPU scatter_max: running max initialised to lowest(), strict '>'
      // (first arg-max wins), untouched outputs filled with 0.
      float m = -3.402823466e+38f;
      int32_t am = -1;
      for (int32_t j = b; j < e; ++j) {
        const int64_t i = gperm[j];
        const float v = x[i * ldx + c];
        if (v > m) {
          m = v;
          am = (int32_t)i;
        }
      }
      out[(int64_t)g * C + c] = am < 0 ? 0.f : m;
      argmax[(int64_t)g * C + c] = am;
    } else {
      float s = 0.f;
      for (int32_t j = b; j < e; ++j) s += x[(int64_t)gperm[j] * ldx + c];
      if (kind == 0) s = s / (float)max(e - b, 1);
      out[(int64_t)g * C + c] = s;
    }
  }
}

__global__ __launch_bounds__(kSegThreads) void k_segpool_bwd(int kind, const float* __restrict__ dout, int64_t C,
                                                              const int32_t* __restrict__ gptr,
                                                              const int32_t* __restrict__ gperm,
                                                              const int32_t* __restrict__ argmax,
                                                              float* __restrict__ dx, int64_t lddx) {
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  const float inv = kind == 0 ? 1.f / (float)max(e - b, 1) : 1.f;
  for (int64_t c = threadIdx.x; c < C; c += kSegThreads) {
    const float d = dout[(int64_t)g * C + c];
    const int32_t am = kind == 1 ? argmax[(int64_t)g * C + c] : -1;
    for (int32_t j = b; j < e; ++j) {
      const int64_t i = gperm[j];
      float v;
      if (kind == 1)
        v = (i == am) ? d : 0.f;
      else
        v = kind == 0 ? d * inv : d;
      dx[i * lddx + c] = v;
    }
  }
}

// Channel slices per workgroup (S) and register rows per wave (R) for a width: C <= 256 -> one
// slice, 8 rows per wave (32-atom chunks: all of QM9 in one); C <= 512 -> 2 slices, 16 rows per
// wave (64-atom chunks); C <= 1024 -> 4 slices (1024 threads, 128 VGPRs), 12 rows per wave (48-atom
// chunks: the synthetic 40-atom molecules in one).
// C > 1024 runs the general body inside the S = 4 instantiation.
int pool_slices(int64_t C) { return C <= 256 ? 1 : (C <= 512 ? 2 : 4); }

template <int S, int P, int R>
void launch_attn_fwd(int H, unsigned G, hipStream_t st, const float* x, int64_t ldx, int64_t N, int64_t C,
                     const float* W, const float* b, const float* tau, const int32_t* gptr, const int32_t* gperm,
                     float* pooled, float* attn, float* scores) {
  const dim3 block(S * P * 64);
  if (H <= 4)
    hipLaunchKernelGGL((k_attn_fwd<S, P, R, 4>), dim3(G), block, 0, st, x, ldx, N, C, W, b, tau, H, gptr, gperm, pooled,
                       attn, scores);
  else
    hipLaunchKernelGGL((k_attn_fwd<S, P, R, 8>), dim3(G), block, 0, st, x, ldx, N, C, W, b, tau, H, gptr, gperm, pooled,
                       attn, scores);
}

template <int S, int P, int R>
void launch_attn_bwd(int H, unsigned G, hipStream_t st, const float* x, int64_t ldx, int64_t N, int64_t C,
                     const float* W, const float* tau, const int32_t* gptr, const int32_t* gperm, const float* attn,
                     const float* scores, const float* dpool, const float* dattn, float* dx, int64_t lddx,
                     float* dW_part, double* db_part, double* dtau_part, double* ds_glob, int32_t* red_cnt,
                     int n_red_cnt) {
  const dim3 block(S * P * 64);
  if (H <= 4)
    hipLaunchKernelGGL((k_attn_bwd<S, P, R, 4>), dim3(G), block, 0, st, x, ldx, N, C, W, tau, H, gptr, gperm, attn,
                       scores, dpool, dattn, dx, lddx, dW_part, db_part, dtau_part, ds_glob, red_cnt, n_red_cnt);
  else
    hipLaunchKernelGGL((k_attn_bwd<S, P, R, 8>), dim3(G), block, 0, st, x, ldx, N, C, W, tau, H, gptr, gperm, attn,
                       scores, dpool, dattn, dx, lddx, dW_part, db_part, dtau_part, ds_glob, red_cnt, n_red_cnt);
}

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" size_t aimx_attn_pool_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t G) {
  return sizeof(float) * (size_t)(G * H * C + 32) +
         sizeof(double) * (size_t)(G * H + G + 2 * H * N + cdiv(G, kRedSlice) * (H * C + H + 1) + 40) +
         sizeof(int32_t) * (size_t)(cdiv(H * C + H + 1, 64) + 16);
}

extern "C" int aimx_attn_pool_forward(const float* x, int64_t ldx, int64_t N, int64_t C, const float* W, const float* b,
                                      const float* tau, int64_t H, const int32_t* gptr, const int32_t* gperm, int64_t G,
                                      float* pooled, float* attn, float* scores, aimx_stream_t s) {
  if (H < 1 || H > kMaxH || C < 0 || N < 0 || G < 0) return AIMX_EARG;
  if (G == 0) return AIMX_OK;
  hipStream_t st = (hipStream_t)s;
  switch (pool_slices(C)) {
    case 1: launch_attn_fwd<1, 4, 8>((int)H, (unsigned)G, st, x, ldx, N, C, W, b, tau, gptr, gperm, pooled, attn, scores); break;
    case 2: launch_attn_fwd<2, 4, 12>((int)H, (unsigned)G, st, x, ldx, N, C, W, b, tau, gptr, gperm, pooled, attn, scores); break;
    default: launch_attn_fwd<4, 2, 24>((int)H, (unsigned)G, st, x, ldx, N, C, W, b, tau, gptr, gperm, pooled, attn, scores);
  }
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_attn_pool_backward(const float* x, int64_t ldx, int64_t N, int64_t C, const float* W,
                                       const float* tau, int64_t H, const int32_t* gptr, const int32_t* gperm,
                                       int64_t G, const float* attn, const float* scores, const float* d_pooled,
                                       const float* d_attn, float* dx, int64_t lddx, float* dW, float* db,
                                       float* dtau, void* ws, size_t ws_bytes, aimx_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (H < 1 || H > kMaxH || C < 0 || N < 0 || G < 0) return AIMX_EARG;
  if (ws_bytes < aimx_attn_pool_workspace_bytes(N, C, H, G) || !ws) return AIMX_EARG;
  float* dW_part = (float*)ws;
  // per-molecule db / dtau partials in fp64: these scalars sum contributions of both signs over
  // all molecules, and fp32 partials left their rounding amplified in the total
  double* db_part = (double*)(((uintptr_t)(dW_part + G * H * C) + 63) & ~(uintptr_t)63);
  double* dtau_part = db_part + G * H;
  double* ds_glob = (double*)(((uintptr_t)(dtau_part + G) + 63) & ~(uintptr_t)63);
  double* slab = (double*)(((uintptr_t)(ds_glob + 2 * H * N) + 63) & ~(uintptr_t)63);
  const int64_t tot = H * C + H + 1, n_slices = std::max<int64_t>(1, cdiv(G, kRedSlice));
  int32_t* red_cnt = (int32_t*)(((uintptr_t)(slab + n_slices * tot) + 63) & ~(uintptr_t)63);
  const int n_red_cnt = (int)cdiv(tot, 64);
  if (G > 0) {
    switch (pool_slices(C)) {
      case 1:
        launch_attn_bwd<1, 4, 8>((int)H, (unsigned)G, s, x, ldx, N, C, W, tau, gptr, gperm, attn, scores, d_pooled, d_attn,
                              dx, lddx, dW_part, db_part, dtau_part, ds_glob, red_cnt, n_red_cnt);
        break;
      case 2:
        launch_attn_bwd<2, 4, 12>((int)H, (unsigned)G, s, x, ldx, N, C, W, tau, gptr, gperm, attn, scores, d_pooled,
                               d_attn, dx, lddx, dW_part, db_part, dtau_part, ds_glob, red_cnt, n_red_cnt);
        break;
      default:
        launch_attn_bwd<4, 2, 24>((int)H, (unsigned)G, s, x, ldx, N, C, W, tau, gptr, gperm, attn, scores, d_pooled,
                               d_attn, dx, lddx, dW_part, db_part, dtau_part, ds_glob, red_cnt, n_red_cnt);
    }
    AIMX_CHECK_LAUNCH();
  }
  static const bool two_launch = tune_i64("AIMX_ATTN_RED2", 0) != 0;  // tuning build: the two-launch reduction
  if (G > 0 && !two_launch) {
    hipLaunchKernelGGL(k_attn_reduce, dim3((unsigned)n_red_cnt, (unsigned)n_slices), dim3(256), 0, s, G, (int)H, C,
                       dW_part, db_part, dtau_part, slab, red_cnt, dW, db, dtau);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  }
  hipLaunchKernelGGL(k_attn_reduce1, dim3((unsigned)cdiv(tot, 64), (unsigned)n_slices), dim3(256), 0, s, G, (int)H, C,
                     dW_part, db_part, dtau_part, slab);
  AIMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_attn_reduce2, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, s, n_slices, (int)H, C, slab, dW,
                     db, dtau);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_segment_pool_forward(int32_t kind, const float* x, int64_t ldx, int64_t N, int64_t C,
                                         const int32_t* gptr, const int32_t* gperm, int64_t G, float* out,
                                         int32_t* argmax, aimx_stream_t s) {
  if (kind < 0 || kind > 2 || (kind == 1 && !argmax) || G < 0 || C < 0) return AIMX_EARG;
  if (G == 0 || C == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_segpool_fwd, dim3((unsigned)G), dim3(kSegThreads), 0, (hipStream_t)s, (int)kind, x, ldx, C,
                     gptr, gperm, out, argmax);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_segment_pool_backward(int32_t kind, const float* dout, int64_t N, int64_t C, const int32_t* gptr,
                                          const int32_t* gperm, int64_t G, const int32_t* argmax, float* dx,
                                          int64_t lddx, aimx_stream_t s) {
  if (kind < 0 || kind > 2 || (kind == 1 && !argmax) || G < 0 || C < 0) return AIMX_EARG;
  if (G == 0 || C == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_segpool_bwd, dim3((unsigned)G), dim3(kSegThreads), 0, (hipStream_t)s, (int)kind, dout, C, gptr,
                     gperm, argmax, dx, lddx);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
