// Partial-charge equilibration, one molecule per workgroup (reference src/models/gnn.py:622-658).
//
//   q = x[:,0], fc = max(x[:,1], 1e-6)
//   Q_g = sum_{i in g} q_i, F_g = max(sum fc_i + 1e-6, 1e-6), dQ_g = total_charge_g - Q_g
//   x' = [q + (fc/F_g) * dQ_g, fc/F_g, x[:,2:]]
// The per-molecule sums run sequentially in atom order in one lane, reproducing the reference's
// zeros(G,1).scatter_add(...) order; the elementwise update is spread over the workgroup.
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

__global__ __launch_bounds__(256) void k_charge_fwd(const float* __restrict__ x, int64_t ldx, int64_t D,
                                                     const int32_t* __restrict__ gptr,
                                                     const int32_t* __restrict__ gperm,
                                                     const float* __restrict__ tc, float* __restrict__ out,
                                                     int64_t ldo) {
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  __shared__ float s_F, s_dQ;
  if (threadIdx.x == 0) {
    float Q = 0.f, Fs = 0.f;
    for (int32_t j = b; j < e; ++j) {
      const int64_t i = gperm[j];
      Q += x[i * ldx];
      Fs += fmaxf(x[i * ldx + 1], 1e-6f);
    }
    s_F = fmaxf(Fs + 1e-6f, 1e-6f);
    s_dQ = tc[g] - Q;
  }
  __syncthreads();
  const float F = s_F, dQ = s_dQ;
  const int64_t n = e - b;
  for (int64_t t = threadIdx.x; t < n * D; t += blockDim.x) {
    const int64_t j = t / D, d = t - j * D;
    const int64_t i = gperm[b + j];
    float v;
    if (d == 0) {
      const float fnew = fmaxf(x[i * ldx + 1], 1e-6f) / F;
      v = x[i * ldx] + fnew * dQ;
    } else if (d == 1) {
      v = fmaxf(x[i * ldx + 1], 1e-6f) / F;
    } else {
      v = x[i * ldx + d];
    }
    out[i * ldo + d] = v;
  }
}

__global__ __launch_bounds__(256) void k_charge_bwd(const float* __restrict__ x, int64_t ldx, int64_t D,
                                                     const int32_t* __restrict__ gptr,
                                                     const int32_t* __restrict__ gperm,
                                                     const float* __restrict__ tc, const float* __restrict__ dout,
                                                     int64_t ldd, float* __restrict__ dx, int64_t lddx) {
  const int g = blockIdx.x;
  const int32_t b = gptr[g], e = gptr[g + 1];
  __shared__ float s_F, s_dQ, s_S1, s_dFu;
  if (threadIdx.x == 0) {
    float Q = 0.f, Fs = 0.f;
    for (int32_t j = b; j < e; ++j) {
      const int64_t i = gperm[j];
      Q += x[i * ldx];
      Fs += fmaxf(x[i * ldx + 1], 1e-6f);
    }
    const float Fpre = Fs + 1e-6f;
    const float F = fmaxf(Fpre, 1e-6f);
    const float dQ = tc[g] - Q;
    // S1 = dL/d(dQ) = sum dq'_i f'_i ; dL/dF = -sum (df'_i + dq'_i dQ) fc_i / F^2
    float S1 = 0.f, SF = 0.f;
    for (int32_t j = b; j < e; ++j) {
      const int64_t i = gperm[j];
      const float fc = fmaxf(x[i * ldx + 1], 1e-6f);
      const float fn = fc / F;
      const float gq = dout[i * ldd], gf = dout[i * ldd + 1];
      S1 += gq * fn;
      SF += (gf + gq * dQ) * fc;
    }
    s_F = F;
    s_dQ = dQ;
    s_S1 = S1;
    s_dFu = (Fpre >= 1e-6f) ? -SF / (F * F) : 0.f;
  }
  __syncthreads();
  const float F = s_F, dQ = s_dQ, S1 = s_S1, dFu = s_dFu;
  const int64_t n = e - b;
  for (int64_t t = threadIdx.x; t < n * D; t += blockDim.x) {
    const int64_t j = t / D, d = t - j * D;
    const int64_t i = gperm[b + j];
    float v;
    if (d == 0) {
      v = dout[i * ldd] - S1;
    } else if (d == 1) {
      const float f = x[i * ldx + 1];
      const float gq = dout[i * ldd], gf = dout[i * ldd + 1];
      const float dfc = (gf + gq * dQ) / F + dFu;
      v = (f >= 1e-6f) ? dfc : 0.f;
    } else {
      v = dout[i * ldd + d];
    }
    dx[i * lddx + d] = v;
  }
}

}  // namespace

int launch_charge_fwd(const float* x, int64_t ldx, int64_t N, int64_t D, const int32_t* gptr, const int32_t* gperm,
                      int64_t G, const float* tc, float* out, int64_t ldo, hipStream_t s) {
  if (D < 2 || G < 0 || N < 0) return AIMX_EARG;
  if (G == 0 || N == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_charge_fwd, dim3((unsigned)G), dim3(256), 0, s, x, ldx, D, gptr, gperm, tc, out, ldo);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

int launch_charge_bwd(const float* x, int64_t ldx, int64_t N, int64_t D, const int32_t* gptr, const int32_t* gperm,
                      int64_t G, const float* tc, const float* dout, int64_t ldd, float* dx, int64_t lddx,
                      hipStream_t s) {
  if (D < 2 || G < 0 || N < 0) return AIMX_EARG;
  if (G == 0 || N == 0) return AIMX_OK;
  hipLaunchKernelGGL(k_charge_bwd, dim3((unsigned)G), dim3(256), 0, s, x, ldx, D, gptr, gperm, tc, dout, ldd, dx,
                     lddx);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

}  // namespace aimx

extern "C" int aimx_partial_charge_forward(const float* x, int64_t ldx, int64_t N, int64_t D, const int32_t* gptr,
                                           const int32_t* gperm, int64_t G, const float* tc, float* out, int64_t ldo,
                                           aimx_stream_t s) {
  return aimx::launch_charge_fwd(x, ldx, N, D, gptr, gperm, G, tc, out, ldo, (hipStream_t)s);
}

extern "C" int aimx_partial_charge_backward(const float* x, int64_t ldx, int64_t N, int64_t D, const int32_t* gptr,
                                            const int32_t* gperm, int64_t G, const float* tc, const float* dout,
                                            int64_t ldd, float* dx, int64_t lddx, aimx_stream_t s) {
  return aimx::launch_charge_bwd(x, ldx, N, D, gptr, gperm, G, tc, dout, ldd, dx, lddx, (hipStream_t)s);
}
