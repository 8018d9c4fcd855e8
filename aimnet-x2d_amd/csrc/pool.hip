// Graph pooling kernels: multi-head attention pool and mean/max/sum, one molecule per workgroup.
//
// Reference: MultiHeadAttentionPoolingLayer.forward, src/models/pooling.py:122-172, and
// Mean/Max/SumPoolingLayer, pooling.py:15-80 (torch_scatter scatter_softmax / scatter_sum /
// scatter_mean / scatter_max). The reference materialises [H, N, hidden] (x expanded per head,
// pooling.py:150-159); here x rows are read once for the H score dot-products (a wave per atom,
// lanes over channels, butterfly reduction) and once more (L2-resident, same molecule) for the
// head-weighted segment sum. Softmax statistics live in LDS. Molecules never span workgroups, so
// there are no atomics; weight gradients are per-molecule partial slabs reduced in molecule order
// by a second kernel (deterministic).
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kMaxH = 8;
constexpr int kCap = 1024;  // atoms per molecule kept in LDS (larger molecules use global scratch)
constexpr int kCapB = 512;  // the same for the backward's fp64 scratch

__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ float block_reduce_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int i = 1; i < kWaves; ++i) s = fmaxf(s, red[i]);
  return s;
}

// Per-(head, atom) scratch for one molecule: LDS image [H][kCap] when the molecule fits, else the
// global [H][N] arrays. Two inlined instantiations keep every access in one address space.
template <bool LDS, typename T = float, int CAP = kCap>
struct Slot {
  T* p;
  int64_t N;
  __device__ __forceinline__ T& at(int h, int j, int64_t i) const { return LDS ? p[h * CAP + j] : p[h * N + i]; }
};

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double block_reduce_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) s += red[i];
  return s;
}

template <bool LDS>
__device__ __forceinline__ void attn_fwd_body(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, const float* __restrict__ bias, float tau,
                                              int H, int32_t b, int n, const int32_t* __restrict__ gperm, int g,
                                              float* __restrict__ pooled, float* __restrict__ attn,
                                              float* __restrict__ scores, Slot<LDS> sa, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // 1) scores s[h,i] = (x_i . W_h + b_h) / tau  (a wave per atom, lanes over channels)
  for (int j = w; j < n; j += kWaves) {
    const int64_t i = gperm[b + j];
    float acc[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) acc[h] = 0.f;
    for (int64_t c = lane; c < C; c += 64) {
      const float xv = x[i * ldx + c];
#pragma unroll
      for (int h = 0; h < kMaxH; ++h)
        if (h < H) acc[h] += xv * W[h * C + c];
    }
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) {
      if (h < H) {
        const float s = (wave_sum(acc[h]) + bias[h]) / tau;
        if (lane == 0) {
          scores[h * N + i] = s;
          if (LDS) sa.at(h, j, i) = s;
        }
      }
    }
  }
  if (!LDS) __threadfence();
  __syncthreads();
  // 2) per-head softmax over the molecule's atoms (torch_scatter.scatter_softmax)
  for (int h = 0; h < H; ++h) {
    float mx = -INFINITY;
    for (int j = threadIdx.x; j < n; j += kThreads) mx = fmaxf(mx, LDS ? sa.at(h, j, 0) : scores[h * N + gperm[b + j]]);
    mx = block_reduce_max(mx, red);
    float sum = 0.f;
    for (int j = threadIdx.x; j < n; j += kThreads)
      sum += expf((LDS ? sa.at(h, j, 0) : scores[h * N + gperm[b + j]]) - mx);
    sum = block_reduce_sum(sum, red);
    for (int j = threadIdx.x; j < n; j += kThreads) {
      const int64_t i = gperm[b + j];
      const float a = expf((LDS ? sa.at(h, j, i) : scores[h * N + i]) - mx) / sum;
      attn[h * N + i] = a;
      if (LDS) sa.at(h, j, i) = a;
    }
  }
  if (!LDS) __threadfence();
  __syncthreads();
  // 3) pooled[g,c] = (sum_h sum_i a[h,i] x[i,c]) / H  (pooling.py:150-161: per-head sums, head mean)
  for (int64_t c = threadIdx.x; c < C; c += kThreads) {
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

// ---- Small-molecule fast path (every QM9 molecule): the molecule's x rows are staged in LDS once
// with 16-B loads (one round trip), then scores, softmax and the pooled sum run from LDS with no
// further global loads; the softmax of head h is one wave's job (lanes over atoms, no barriers).
// Same arithmetic per value as the general body above, except the softmax max/sum reductions,
// which run as one wave butterfly instead of a block reduction (fp32 reassociation only).
constexpr int kFastAtoms = 64;             // atoms per molecule (one wave's lanes in the softmax)
constexpr int kFastXBytes = 32 * 1024;     // LDS for the staged rows
constexpr int kSmemBytes = kFastXBytes + 8 * 1024;
static_assert(kMaxH * kCap * 4 <= kSmemBytes && kMaxH * kCapB * 8 <= kSmemBytes, "general-path scratch fits");

__device__ __forceinline__ bool fast_ok(int n, int64_t C, int H) {
  return n <= kFastAtoms && (int64_t)n * C * 4 <= kFastXBytes && H <= kMaxH && (C % 4) == 0;
}

// head weights [H][C] staged after the fast path's sa scratch (16-B aligned: W 16-B aligned too)
__device__ __forceinline__ bool wlds_ok(int64_t C, int H) {
  return (int64_t)H * C * 4 + kMaxH * kFastAtoms * 4 <= kSmemBytes - kFastXBytes && (C % 4) == 0;
}

// stage rows gperm[b .. b+n) of x into xs[n][C] (16-B loads; ldx % 4 == 0 checked by the host)
__device__ __forceinline__ void stage_rows(const float* __restrict__ x, int64_t ldx, int64_t C, int32_t b, int n,
                                           const int32_t* __restrict__ gperm, float* xs) {
  const int c4 = (int)(C / 4);
  const int tot = n * c4;
  for (int q = threadIdx.x; q < tot; q += kThreads) {
    const int j = q / c4, c = (q - j * c4) * 4;
    const int64_t i = gperm[b + j];
    *reinterpret_cast<float4*>(xs + j * C + c) = *reinterpret_cast<const float4*>(x + i * ldx + c);
  }
}

__device__ __forceinline__ void attn_fwd_fast(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, const float* __restrict__ bias, float tau,
                                              int H, int32_t b, int n, const int32_t* __restrict__ gperm, int g,
                                              float* __restrict__ pooled, float* __restrict__ attn,
                                              float* __restrict__ scores, char* smem) {
  float* xs = reinterpret_cast<float*>(smem);                      // [n][C]
  float* sa = reinterpret_cast<float*>(smem + kFastXBytes);        // [kMaxH][kFastAtoms]
  float* ws = sa + kMaxH * kFastAtoms;                             // [H][C] when it fits
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // the head weights are read once per atom by every wave: stage them beside the rows (one
  // round trip for both) when they fit the scratch after sa, else read them from global memory
  const bool wlds = wlds_ok(C, H) && ((uintptr_t)W & 15) == 0;
  if (wlds)
    for (int q = threadIdx.x; q < H * (int)C / 4; q += kThreads)
      *reinterpret_cast<float4*>(ws + 4 * q) = *reinterpret_cast<const float4*>(W + 4 * q);
  stage_rows(x, ldx, C, b, n, gperm, xs);
  __syncthreads();
  const float* Wr = wlds ? ws : W;
  // 1) scores: a wave per atom, lanes over channels (same order as attn_fwd_body)
  for (int j = w; j < n; j += kWaves) {
    float acc[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) acc[h] = 0.f;
    for (int64_t c = lane; c < C; c += 64) {
      const float xv = xs[j * C + c];
#pragma unroll
      for (int h = 0; h < kMaxH; ++h)
        if (h < H) acc[h] += xv * Wr[h * C + c];
    }
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) {
      if (h < H) {
        const float sc = (wave_sum(acc[h]) + bias[h]) / tau;
        if (lane == 0) {
          scores[h * N + gperm[b + j]] = sc;
          sa[h * kFastAtoms + j] = sc;
        }
      }
    }
  }
  __syncthreads();
  // 2) softmax of head h by wave h % kWaves, lanes over atoms
  for (int h = w; h < H; h += kWaves) {
    const float v = lane < n ? sa[h * kFastAtoms + lane] : -INFINITY;
    const float mx = wave_max(v);
    const float ex = lane < n ? expf(v - mx) : 0.f;
    const float sum = wave_sum(ex);
    if (lane < n) {
      const float a = expf(v - mx) / sum;
      attn[h * N + gperm[b + lane]] = a;
      sa[h * kFastAtoms + lane] = a;
    }
  }
  __syncthreads();
  // 3) pooled[g,c] = (sum_h sum_i a[h,i] x[i,c]) / H
  for (int64_t c = threadIdx.x; c < C; c += kThreads) {
    float acc[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) acc[h] = 0.f;
    for (int j = 0; j < n; ++j) {
      const float xv = xs[j * C + c];
#pragma unroll
      for (int h = 0; h < kMaxH; ++h)
        if (h < H) acc[h] += sa[h * kFastAtoms + j] * xv;
    }
    float sm = 0.f;
#pragma unroll
    for (int h = 0; h < kMaxH; ++h)
      if (h < H) sm += acc[h];
    pooled[(int64_t)g * C + c] = sm / (float)H;
  }
}

__global__ __launch_bounds__(kThreads) void k_attn_fwd(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                                        const float* __restrict__ W, const float* __restrict__ bias,
                                                        const float* __restrict__ tau_p, int H,
                                                        const int32_t* __restrict__ gptr,
                                                        const int32_t* __restrict__ gperm, float* __restrict__ pooled,
                                                        float* __restrict__ attn, float* __restrict__ scores) {
  __shared__ __attribute__((aligned(16))) char smem[kSmemBytes];
  __shared__ float red[kWaves];
  float* sa = reinterpret_cast<float*>(smem);  // general path: [kMaxH][kCap] floats
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  const int n = e - b;
  const float tau = *tau_p;
  if (fast_ok(n, C, H) && (ldx % 4) == 0 && ((uintptr_t)x & 15) == 0)
    attn_fwd_fast(x, ldx, N, C, W, bias, tau, H, b, n, gperm, g, pooled, attn, scores, smem);
  else if (n <= kCap)
    attn_fwd_body<true>(x, ldx, N, C, W, bias, tau, H, b, n, gperm, g, pooled, attn, scores, Slot<true>{sa, N}, red);
  else
    attn_fwd_body<false>(x, ldx, N, C, W, bias, tau, H, b, n, gperm, g, pooled, attn, scores, Slot<false>{attn, N},
                         red);
}

// Backward. ds[h,i] = a (da - sum_j a da), da[h,i] = (x_i . dpooled[g]) / H + d_attn[h,i].
// The softmax backward cancels (da - <a, da>) when a molecule's attention is peaked, so every
// reduction here (dots, <a, da>, ds, the dW/db/dtau partial sums) is accumulated in fp64: the
// kernel is memory/latency-bound and the fp64 VALU rate is not the limit.
template <bool LDS>
__device__ __forceinline__ void attn_bwd_body(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, float tau, int H, int32_t b, int n,
                                              const int32_t* __restrict__ gperm, int g,
                                              const float* __restrict__ attn, const float* __restrict__ scores,
                                              const float* __restrict__ dpool, const float* __restrict__ dattn,
                                              float* __restrict__ dx, int64_t lddx, float* __restrict__ dW_part,
                                              float* __restrict__ db_part, float* __restrict__ dtau_part,
                                              Slot<LDS, double, kCapB> sds, double* red) {
  const double invH = 1.0 / (double)H;
  const double dtau_inv = 1.0 / (double)tau;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* q = dpool + (int64_t)g * C;
  // 1) da[h,i]
  for (int j = w; j < n; j += kWaves) {
    const int64_t i = gperm[b + j];
    double acc = 0.0;
    for (int64_t c = lane; c < C; c += 64) acc += (double)x[i * ldx + c] * (double)q[c];
    const double d = wave_sum_d(acc) * invH;
    if (lane < H) sds.at(lane, j, i) = d + (dattn ? (double)dattn[lane * N + i] : 0.0);
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
    for (int j = threadIdx.x; j < n; j += kThreads) {
      const int64_t i = gperm[b + j];
      const double a = attn[h * N + i];
      t += a * sds.at(h, j, i);
      asum += a;
    }
    t = block_reduce_sum_d(t, red);
    asum = block_reduce_sum_d(asum, red);
    if (asum > 0.0) t /= asum;
    double dbs = 0.0;
    for (int j = threadIdx.x; j < n; j += kThreads) {
      const int64_t i = gperm[b + j];
      const double ds = (double)attn[h * N + i] * (sds.at(h, j, i) - t);
      sds.at(h, j, i) = ds;
      dbs += ds;
      dtau_acc += ds * (double)scores[h * N + i];
    }
    dbs = block_reduce_sum_d(dbs, red);
    if (threadIdx.x == 0) db_part[(int64_t)g * H + h] = (float)(dbs * dtau_inv);
  }
  dtau_acc = block_reduce_sum_d(dtau_acc, red);
  if (threadIdx.x == 0) dtau_part[g] = (float)(-dtau_acc * dtau_inv);
  if (!LDS) __threadfence();
  __syncthreads();
  // 3) dx_i = (sum_h a[h,i]) q / H + sum_h ds[h,i] W_h / tau ; dW_part[g,h] = sum_i ds[h,i] x_i / tau
  for (int64_t c = threadIdx.x; c < C; c += kThreads) {
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

__device__ __forceinline__ void attn_bwd_fast(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                              const float* __restrict__ W, float tau, int H, int32_t b, int n,
                                              const int32_t* __restrict__ gperm, int g,
                                              const float* __restrict__ attn, const float* __restrict__ scores,
                                              const float* __restrict__ dpool, const float* __restrict__ dattn,
                                              float* __restrict__ dx, int64_t lddx, float* __restrict__ dW_part,
                                              float* __restrict__ db_part, float* __restrict__ dtau_part, char* smem,
                                              double* red) {
  float* xs = reinterpret_cast<float*>(smem);                                // [n][C]
  double* sds = reinterpret_cast<double*>(smem + kFastXBytes);               // [kMaxH][kFastAtoms]
  float* sa = reinterpret_cast<float*>(smem + kFastXBytes + 8 * kMaxH * kFastAtoms);
  float* ssc = sa + kMaxH * kFastAtoms;
  const double invH = 1.0 / (double)H;
  const double dtau_inv = 1.0 / (double)tau;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* q = dpool + (int64_t)g * C;
  stage_rows(x, ldx, C, b, n, gperm, xs);
  for (int t = threadIdx.x; t < H * n; t += kThreads) {
    const int h = t / n, j = t - h * n;
    const int64_t i = gperm[b + j];
    sa[h * kFastAtoms + j] = attn[h * N + i];
    ssc[h * kFastAtoms + j] = scores[h * N + i];
  }
  __syncthreads();
  // 1) da[h,i] (a wave per atom, lanes over channels, fp64 as in attn_bwd_body)
  for (int j = w; j < n; j += kWaves) {
    double acc = 0.0;
    for (int64_t c = lane; c < C; c += 64) acc += (double)xs[j * C + c] * (double)q[c];
    const double d = wave_sum_d(acc) * invH;
    if (lane < H) sds[lane * kFastAtoms + j] = d + (dattn ? (double)dattn[lane * N + gperm[b + j]] : 0.0);
  }
  __syncthreads();
  // 2) ds = a (da - <a, da> / sum a) per head (wave h % kWaves, lanes over atoms); db, dtau partials
  double dtau_acc = 0.0;
  for (int h = w; h < H; h += kWaves) {
    const bool in = lane < n;
    const double a = in ? (double)sa[h * kFastAtoms + lane] : 0.0;
    const double da = in ? sds[h * kFastAtoms + lane] : 0.0;
    double t = wave_sum_d(a * da);
    const double asum = wave_sum_d(a);
    if (asum > 0.0) t /= asum;
    const double ds = a * (da - t);
    if (in) sds[h * kFastAtoms + lane] = ds;
    const double dbs = wave_sum_d(ds);
    if (lane == 0) db_part[(int64_t)g * H + h] = (float)(dbs * dtau_inv);
    dtau_acc += ds * (in ? (double)ssc[h * kFastAtoms + lane] : 0.0);
  }
  dtau_acc = block_reduce_sum_d(dtau_acc, red);
  if (threadIdx.x == 0) dtau_part[g] = (float)(-dtau_acc * dtau_inv);
  __syncthreads();
  // 3) dx_i = (sum_h a[h,i]) q / H + sum_h ds[h,i] W_h / tau ; dW_part[g,h] = sum_i ds[h,i] x_i / tau
  for (int64_t c = threadIdx.x; c < C; c += kThreads) {
    const double qc = (double)q[c] * invH;
    double wc[kMaxH], dw[kMaxH];
#pragma unroll
    for (int h = 0; h < kMaxH; ++h) {
      wc[h] = h < H ? (double)W[h * C + c] : 0.0;
      dw[h] = 0.0;
    }
    for (int j = 0; j < n; ++j) {
      const double xv = xs[j * C + c];
      double asum = 0.0, dsw = 0.0;
#pragma unroll
      for (int h = 0; h < kMaxH; ++h) {
        if (h < H) {
          const double ds = sds[h * kFastAtoms + j];
          asum += sa[h * kFastAtoms + j];
          dsw += ds * wc[h];
          dw[h] += ds * xv;
        }
      }
      dx[gperm[b + j] * lddx + c] = (float)(asum * qc + dsw * dtau_inv);
    }
#pragma unroll
    for (int h = 0; h < kMaxH; ++h)
      if (h < H) dW_part[((int64_t)g * H + h) * C + c] = (float)(dw[h] * dtau_inv);
  }
}

__global__ __launch_bounds__(kThreads) void k_attn_bwd(const float* __restrict__ x, int64_t ldx, int64_t N, int64_t C,
                                                        const float* __restrict__ W, const float* __restrict__ tau_p,
                                                        int H, const int32_t* __restrict__ gptr,
                                                        const int32_t* __restrict__ gperm,
                                                        const float* __restrict__ attn, const float* __restrict__ scores,
                                                        const float* __restrict__ dpool,
                                                        const float* __restrict__ dattn, float* __restrict__ dx,
                                                        int64_t lddx, float* __restrict__ dW_part,
                                                        float* __restrict__ db_part, float* __restrict__ dtau_part,
                                                        double* __restrict__ ds_glob) {
  __shared__ __attribute__((aligned(16))) char smem[kSmemBytes];
  __shared__ double red[kWaves];
  double* sds = reinterpret_cast<double*>(smem);  // general path: [kMaxH][kCapB] doubles
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  const int n = e - b;
  const float tau = *tau_p;
  if (fast_ok(n, C, H) && (ldx % 4) == 0 && ((uintptr_t)x & 15) == 0)
    attn_bwd_fast(x, ldx, N, C, W, tau, H, b, n, gperm, g, attn, scores, dpool, dattn, dx, lddx, dW_part, db_part,
                  dtau_part, smem, red);
  else if (n <= kCapB)
    attn_bwd_body<true>(x, ldx, N, C, W, tau, H, b, n, gperm, g, attn, scores, dpool, dattn, dx, lddx, dW_part, db_part,
                        dtau_part, Slot<true, double, kCapB>{sds, N}, red);
  else
    attn_bwd_body<false>(x, ldx, N, C, W, tau, H, b, n, gperm, g, attn, scores, dpool, dattn, dx, lddx, dW_part,
                         db_part, dtau_part, Slot<false, double, kCapB>{ds_glob, N}, red);
}

// One wave per output value (dW[h,c], db[h], dtau): lanes take molecules g = lane, lane+64, ... and
// the 64 partial sums are combined by a fixed butterfly — deterministic and latency-parallel.
__global__ void k_attn_reduce(int64_t G, int H, int64_t C, const float* __restrict__ dW_part,
                              const float* __restrict__ db_part, const float* __restrict__ dtau_part,
                              float* __restrict__ dW, float* __restrict__ db, float* __restrict__ dtau) {
  const int64_t nw = (int64_t)H * C;
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t t = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6); t < nw + H + 1; t += waves) {
    double s = 0.0;
    if (t < nw) {
      for (int64_t g = lane; g < G; g += 64) s += dW_part[g * nw + t];
    } else if (t < nw + H) {
      for (int64_t g = lane; g < G; g += 64) s += db_part[g * H + (t - nw)];
    } else {
      for (int64_t g = lane; g < G; g += 64) s += dtau_part[g];
    }
    s = wave_sum_d(s);
    if (lane == 0) {
      if (t < nw)
        dW[t] = (float)s;
      else if (t < nw + H)
        db[t - nw] = (float)s;
      else
        *dtau = (float)s;
    }
  }
}

// kind: 0 mean, 1 max, 2 sum
__global__ __launch_bounds__(kThreads) void k_segpool_fwd(int kind, const float* __restrict__ x, int64_t ldx, int64_t C,
                                                           const int32_t* __restrict__ gptr,
                                                           const int32_t* __restrict__ gperm, float* __restrict__ out,
                                                           int32_t* __restrict__ argmax) {
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  for (int64_t c = threadIdx.x; c < C; c += kThreads) {
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

__global__ __launch_bounds__(kThreads) void k_segpool_bwd(int kind, const float* __restrict__ dout, int64_t C,
                                                           const int32_t* __restrict__ gptr,
                                                           const int32_t* __restrict__ gperm,
                                                           const int32_t* __restrict__ argmax, float* __restrict__ dx,
                                                           int64_t lddx) {
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  const float inv = kind == 0 ? 1.f / (float)max(e - b, 1) : 1.f;
  for (int64_t c = threadIdx.x; c < C; c += kThreads) {
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

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" size_t aimx_attn_pool_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t G) {
  return sizeof(float) * (size_t)(G * H * C + G * H + G + 64) + sizeof(double) * (size_t)(H * N + 8);
}

extern "C" int aimx_attn_pool_forward(const float* x, int64_t ldx, int64_t N, int64_t C, const float* W, const float* b,
                                      const float* tau, int64_t H, const int32_t* gptr, const int32_t* gperm, int64_t G,
                                      float* pooled, float* attn, float* scores, aimx_stream_t s) {
  if (H < 1 || H > kMaxH || C < 0 || N < 0 || G < 0) return AIMX_EARG;
  if (G == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_attn_fwd, dim3((unsigned)G), dim3(kThreads), 0, (hipStream_t)s, x, ldx, N, C, W, b, tau, (int)H,
                     gptr, gperm, pooled, attn, scores);
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
  float* db_part = dW_part + G * H * C;
  float* dtau_part = db_part + G * H;
  double* ds_glob = (double*)(((uintptr_t)(dtau_part + G) + 63) & ~(uintptr_t)63);
  if (G > 0) {
    hipLaunchKernelGGL(k_attn_bwd, dim3((unsigned)G), dim3(kThreads), 0, s, x, ldx, N, C, W, tau, (int)H, gptr,
                       gperm, attn, scores, d_pooled, d_attn, dx, lddx, dW_part, db_part, dtau_part, ds_glob);
    AIMX_CHECK_LAUNCH();
  }
  const int64_t tot = H * C + H + 1;
  hipLaunchKernelGGL(k_attn_reduce, dim3((unsigned)std::min<int64_t>(cdiv(tot, 4), 4096)), dim3(256), 0, s, G,
                     (int)H, C, dW_part, db_part, dtau_part, dW, db, dtau);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_segment_pool_forward(int32_t kind, const float* x, int64_t ldx, int64_t N, int64_t C,
                                         const int32_t* gptr, const int32_t* gperm, int64_t G, float* out,
                                         int32_t* argmax, aimx_stream_t s) {
  if (kind < 0 || kind > 2 || (kind == 1 && !argmax) || G < 0 || C < 0) return AIMX_EARG;
  if (G == 0 || C == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_segpool_fwd, dim3((unsigned)G), dim3(kThreads), 0, (hipStream_t)s, (int)kind, x, ldx, C, gptr,
                     gperm, out, argmax);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_segment_pool_backward(int32_t kind, const float* dout, int64_t N, int64_t C, const int32_t* gptr,
                                          const int32_t* gperm, int64_t G, const int32_t* argmax, float* dx,
                                          int64_t lddx, aimx_stream_t s) {
  if (kind < 0 || kind > 2 || (kind == 1 && !argmax) || G < 0 || C < 0) return AIMX_EARG;
  if (G == 0 || C == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_segpool_bwd, dim3((unsigned)G), dim3(kThreads), 0, (hipStream_t)s, (int)kind, dout, C, gptr,
                     gperm, argmax, dx, lddx);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
