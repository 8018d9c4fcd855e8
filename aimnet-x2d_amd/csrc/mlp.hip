// Fused node-update MLP of one shell layer: all of the layer's MLP blocks in ONE launch forward
// and ONE launch for the activation-gradient chain backward.
//
// Reference: ShellConvolutionLayer.forward, src/models/layers.py:82-106 (+ the outer residual
// gnn.py:302-306): with a0 = act(u) (u = the input projection, computed by the preceding GEMM)
//   v_k = a_k W1_k^T + b1_k ; r_k = dropout(act(v_k)) ; a_{k+1} = r_k W2_k^T + b2_k + a_k
//   out = a_nm + g (+ x)
// backward, given dY = d out:
//   dA_nm = dY ; dV_k = (dA_{k+1} W2_k) * mask / (1-p) * act'(v_k) ; dA_k = dA_{k+1} + dV_k W1_k
//   du = dA_0 * act'(u) ;  dUG = [du | dY]
// Launched per GEMM these are 2 * nm latency-bound kernels per layer and direction (N = atoms
// rows, D x D weights: ~8-12 us each at c2). Here a workgroup owns 32 atoms: its activations stay
// in LDS for the whole chain, each wave owns 16 output columns (both 16-row tiles, two independent
// MFMA accumulators) and streams its own weight rows through a private LDS slice, so the only
// workgroup barriers are the one per GEMM. Dropout uses the same hash, salt and index as the
// per-GEMM path (hash(seed, layer * nm + k, row * D + col)), so the masks are identical.
#include <algorithm>
#include <cstdlib>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kRT = 1;                 // 16-row tiles per workgroup
constexpr int kRows = 16 * kRT;        // atoms per workgroup
constexpr int kBK = 32;                // k slice
constexpr int kBSt = kBK + 4;          // LDS row stride of a staged weight slice
constexpr int kWS = 16 * kBSt;         // floats of one wave's staging slice
constexpr int kP = 4;                  // weight slices in flight per wave
constexpr int kInitUnroll = 12;        // tile loads in flight per thread at kernel start
constexpr int kMaxWaves = 8;  // <= 512 threads: up to 256 VGPRs per lane (no spills)

__host__ __device__ inline int pad32(int d) { return (d + 31) / 32 * 32; }
__host__ __device__ inline int lds_stride(int d) { return pad32(d) + 4; }  // = 4 mod 32: conflict-free b128

// C[32][N] = A[32][K] . B over a workgroup; A in LDS (row stride lda, zero in columns [K, Kp)).
// B(k, n) = W[n * ldw + k] when KC (k-contiguous: nn.Linear forward) else W[k * ldw + n].
// Wave w owns column fragments cf = w, w + nwaves, ... (16 columns each) for both row tiles.
template <bool KC, class Pre, class Epi>
__device__ __forceinline__ void rows_gemm(const float* A, int lda, int K, const float* W, int64_t ldw, int N,
                                          float* Bs, Pre pre, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int nsl = pad32(K) / kBK;
  const int lr = lane & 15, lq = 4 * (lane >> 4);
  float* Bw = Bs + wave * kWS;
  const int CF = (N + 15) / 16;
  for (int cf = wave; cf < CF; cf += nw) {
    const int n0 = cf * 16;
    // staging sources (clamped: rows/cols past N and k past K read valid finite weights whose
    // products meet zero A columns or land in dropped outputs)
    const float* src[2];
    int dst[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (KC) {
        const int row = 8 * i + (lane >> 3), kq = (lane & 7) * 4;
        src[i] = W + (int64_t)min(n0 + row, N - 1) * ldw + kq;
        dst[i] = row * kBSt + kq;
      } else {
        const int kr = (lane >> 2) + 16 * i, nq = min(n0 + (lane & 3) * 4, N - 4) - n0;
        src[i] = W + (int64_t)kr * ldw + n0 + nq;
        dst[i] = nq * kBSt + kr;  // transposed on the store
      }
    }
    const int col = n0 + lr;
    float2 pv[kRT][4];
#pragma unroll
    for (int t = 0; t < kRT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) pv[t][r] = pre(t * 16 + (lane >> 4) * 4 + r, min(col, N - 1));
    floatx4 acc[kRT];
#pragma unroll
    for (int t = 0; t < kRT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 rg[kP][2];
    auto load = [&](int sl, floatx4 (&r)[2]) {
      const int s = min(sl, nsl - 1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (KC) {
          // k quad past K: clamp to the last full quad (K % 4 == 0 is required on the host)
          const int k = min(s * kBK + (lane & 7) * 4, K - 4) - (lane & 7) * 4;
          r[i] = *reinterpret_cast<const floatx4*>(src[i] + k);
        } else {
          const int k = min(s * kBK + (lane >> 2) + 16 * i, K - 1) - ((lane >> 2) + 16 * i);
          r[i] = *reinterpret_cast<const floatx4*>(src[i] + (int64_t)k * ldw);
        }
      }
    };
#pragma unroll
    for (int q = 0; q < kP; ++q) load(q, rg[q]);
    __builtin_amdgcn_sched_barrier(0);
    const float* b0 = Bw + lr * kBSt + lq;
    for (int s0 = 0; s0 < nsl; s0 += kP) {
#pragma unroll
      for (int q = 0; q < kP; ++q) {
        const int sl = s0 + q;
        if (sl < nsl) {  // uniform
          if (KC) {
#pragma unroll
            for (int i = 0; i < 2; ++i) *reinterpret_cast<floatx4*>(Bw + dst[i]) = rg[q][i];
          } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int e = 0; e < 4; ++e) Bw[dst[i] + e * kBSt] = rg[q][i][e];
          }
          load(sl + kP, rg[q]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const floatx4 b = *reinterpret_cast<const floatx4*>(b0 + 16 * h);
#pragma unroll
            for (int t = 0; t < kRT; ++t) {
              const floatx4 a = *reinterpret_cast<const floatx4*>(A + (t * 16 + lr) * lda + sl * kBK + lq + 16 * h);
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc[t], 0, 0, 0);
            }
          }
        }
      }
    }
    if (col < N) {
#pragma unroll
      for (int t = 0; t < kRT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) epi(t * 16 + (lane >> 4) * 4 + r, col, acc[t][r], pv[t][r]);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float drop_scale(float p) { return p < 1.f ? 1.f / (1.f - p) : 0.f; }

struct MlpFwd {
  int64_t N, D;
  int32_t nm, act, drop, salt0;
  float drop_p;
  const int64_t* seed;
  const float* ug;  // [N, 2D]: a0 = act(u), g
  const float* x;   // outer residual (nullable), ld ldx
  int64_t ldx;
  const float* w1[8];
  const float* b1[8];
  const float* w2[8];
  const float* b2[8];
  float* V[8];
  float* R[8];
  float* A[8];
  uint8_t* M[8];
  float* out;
  int64_t ldo;
};

__global__ __launch_bounds__(512) void k_mlp_fwd(const MlpFwd p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int D = (int)p.D, lda = lds_stride(D), Dp = pad32(D);
  const int nw = blockDim.x >> 6;
  float* Bs = lds;
  float* Xa = lds + nw * kWS;    // current block input a_k   [32][lda]
  float* Hb = Xa + kRows * lda;  // r_k                        [32][lda]
  const int64_t r0 = (int64_t)blockIdx.x * kRows;
  const int64_t N = p.N;
  // all of the tile's loads in flight at once (a plain strided loop issues them one round trip
  // at a time); zero k padding for both A operands
  for (int e0 = 0; e0 < kRows * Dp; e0 += kInitUnroll * (int)blockDim.x) {
    float v[kInitUnroll];
#pragma unroll
    for (int u = 0; u < kInitUnroll; ++u) {
      const int e = e0 + u * blockDim.x + threadIdx.x;
      const int r = e / Dp, c = e - r * Dp;
      const int64_t g = r0 + r;
      const bool ok = e < kRows * Dp && c < D && g < N;
      v[u] = p.ug[(ok ? g * 2 * D + c : 0)];
      v[u] = ok ? v[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kInitUnroll; ++u) {
      const int e = e0 + u * blockDim.x + threadIdx.x;
      if (e < kRows * Dp) {
        const int r = e / Dp, c = e - r * Dp;
        Xa[r * lda + c] = v[u];
        Hb[r * lda + c] = 0.f;
      }
    }
  }
  __syncthreads();
  const float scale = drop_scale(p.drop_p);
  const uint64_t seed = p.drop ? (uint64_t)*p.seed : 0;
  for (int k = 0; k < p.nm; ++k) {
    const bool last = k == p.nm - 1;
    float* V = p.V[k];
    float* R = p.R[k];
    uint8_t* M = p.M[k];
    const float* b1 = p.b1[k];
    const uint32_t salt = (uint32_t)(p.salt0 + k);
    rows_gemm<true>(Xa, lda, D, p.w1[k], D, D, Bs, [&](int, int c) { return make_float2(b1[c], 0.f); },
                    [&](int r, int c, float acc, float2 pv) {
                      const int64_t g = r0 + r;
                      const float v = acc + pv.x;
                      float a = act_fwd(p.act, v);
                      if (p.drop) {
                        const bool keep = hash_uniform(seed, salt, (uint64_t)g * (uint64_t)D + (uint64_t)c) >= p.drop_p;
                        a = keep ? a * scale : 0.f;
                        if (g < N) M[g * D + c] = keep ? 1 : 0;
                      }
                      Hb[r * lda + c] = a;
                      if (g < N) {
                        V[g * D + c] = v;
                        R[g * D + c] = a;
                      }
                    });
    const float* b2 = p.b2[k];
    float* Ak = last ? nullptr : p.A[k];
    // epilogue operands: b2, and for the last block the global skip g (+ outer residual x)
    rows_gemm<true>(Hb, lda, D, p.w2[k], D, D, Bs,
                    [&](int r, int c) {
                      float add = b2[c];
                      if (last) {
                        const int64_t g = min(r0 + r, N - 1);
                        add += p.ug[g * 2 * D + D + c];
                        if (p.x) add += p.x[g * p.ldx + c];
                      }
                      return make_float2(add, 0.f);
                    },
                    [&](int r, int c, float acc, float2 pv) {
                      const int64_t g = r0 + r;
                      // a_{k+1} = r W2^T + b2 + a_k (+ g + x): the GEMM path's epilogue order
                      // (bias, then residuals in argument order) up to fp32 rounding
                      const float a = acc + pv.x + Xa[r * lda + c];
                      Xa[r * lda + c] = a;
                      if (g < N) {
                        if (last)
                          p.out[g * p.ldo + c] = a;
                        else
                          Ak[g * D + c] = a;
                      }
                    });
  }
}

struct MlpBwd {
  int64_t N, D;
  int32_t nm, act, drop;
  float drop_p;
  const float* dy;  // d out [N, D], ld lddy
  int64_t lddy;
  const float* u;   // pre-activation of a0 [N, D]
  const float* w1[8];
  const float* w2[8];
  const float* V[8];
  const uint8_t* M[8];
  float* dV[8];
  float* dA[8];     // dA_k for k = 1..nm-1 (the gradient w.r.t. block k's input), index k - 1
  float* dug;       // [N, 2D]: [du | dY]
};

__global__ __launch_bounds__(512) void k_mlp_bwd(const MlpBwd p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int D = (int)p.D, lda = lds_stride(D), Dp = pad32(D);
  const int nw = blockDim.x >> 6;
  float* Bs = lds;
  float* DA = lds + nw * kWS;    // gradient w.r.t. the current block output   [32][lda]
  float* DV = DA + kRows * lda;  // dV_k                                        [32][lda]
  const int64_t r0 = (int64_t)blockIdx.x * kRows;
  const int64_t N = p.N;
  for (int e0 = 0; e0 < kRows * Dp; e0 += kInitUnroll * (int)blockDim.x) {
    float v[kInitUnroll];
#pragma unroll
    for (int u = 0; u < kInitUnroll; ++u) {
      const int e = e0 + u * blockDim.x + threadIdx.x;
      const int r = e / Dp, c = e - r * Dp;
      const int64_t g = r0 + r;
      const bool ok = e < kRows * Dp && c < D && g < N;
      v[u] = p.dy[(ok ? g * p.lddy + c : 0)];
      v[u] = ok ? v[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kInitUnroll; ++u) {
      const int e = e0 + u * blockDim.x + threadIdx.x;
      if (e < kRows * Dp) {
        const int r = e / Dp, c = e - r * Dp;
        const int64_t g = r0 + r;
        DA[r * lda + c] = v[u];
        DV[r * lda + c] = 0.f;
        if (c < D && g < N) p.dug[g * 2 * D + D + c] = v[u];  // dg = dY
      }
    }
  }
  __syncthreads();
  const float scale = drop_scale(p.drop_p);
  for (int k = p.nm - 1; k >= 0; --k) {
    const float* V = p.V[k];
    const uint8_t* M = p.M[k];
    float* dVk = p.dV[k];
    // dV = (dA W2) * mask/(1-p) * act'(v)
    rows_gemm<false>(DA, lda, D, p.w2[k], D, D, Bs,
                     [&](int r, int c) {
                       const int64_t g = min(r0 + r, N - 1);
                       const float m = p.drop ? (M[g * D + c] ? scale : 0.f) : 1.f;
                       return make_float2(act_grad(p.act, V[g * D + c]), m);
                     },
                     [&](int r, int c, float acc, float2 pv) {
                       const int64_t g = r0 + r;
                       const float dv = (g < N) ? acc * pv.y * pv.x : 0.f;
                       DV[r * lda + c] = dv;
                       if (g < N) dVk[g * D + c] = dv;
                     });
    // dA_k = dA_{k+1} + dV W1 ; for k == 0: du = dA_0 * act'(u)
    float* dAk = k > 0 ? p.dA[k - 1] : nullptr;
    rows_gemm<false>(DV, lda, D, p.w1[k], D, D, Bs,
                     [&](int r, int c) {
                       const int64_t g = min(r0 + r, N - 1);
                       return make_float2(k == 0 ? act_grad(p.act, p.u[g * D + c]) : 1.f, 0.f);
                     },
                     [&](int r, int c, float acc, float2 pv) {
                       const int64_t g = r0 + r;
                       const float da = DA[r * lda + c] + acc;
                       DA[r * lda + c] = da;
                       if (g < N) {
                         if (k > 0)
                           dAk[g * D + c] = da;
                         else
                           p.dug[g * 2 * D + c] = da * pv.x;
                       }
                     });
  }
}

size_t mlp_lds_bytes(int64_t D) {
  const int nw = std::min<int>(kMaxWaves, (int)((D + 15) / 16));
  return sizeof(float) * (size_t)(nw * kWS + 2 * kRows * lds_stride((int)D));
}

int mlp_threads(int64_t D) { return 64 * std::min<int>(kMaxWaves, (int)((D + 15) / 16)); }

bool mlp_lds_ok(int64_t D) {
  static const bool set = [] {
    (void)hipFuncSetAttribute((const void*)k_mlp_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_mlp_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)set;
  return mlp_lds_bytes(D) <= 160 * 1024;
}

}  // namespace

// Opt-in (AIMX_FUSED_MLP=1). Measured at c2 (N = 9.2k atoms, D = 76, MI355X) the fused chain is
// slower than the per-GEMM path it replaces: train step 1148-1182 vs 1110 us (32- and 16-row
// workgroups). Each workgroup walks 2 * nm dependent GEMM phases with only ~1-2 workgroups per CU
// to overlap them, while the per-GEMM kernels spread each phase over ~440 workgroups.
bool mlp_fused_ok(int64_t D, int64_t nm) {
  const char* e = getenv("AIMX_FUSED_MLP");
  return e && atoi(e) == 1 && D >= 4 && D % 4 == 0 && nm >= 1 && nm <= 8 && mlp_lds_ok(D);
}

int launch_mlp_fwd(const AimxShellStack* s, int64_t l, const float* x_res, int64_t ldx, float* out, int64_t ldo,
                   hipStream_t st) {
  MlpFwd p{};
  const int64_t nm = s->num_mlp;
  p.N = s->N;
  p.D = s->D;
  p.nm = (int32_t)nm;
  p.act = s->act;
  p.drop = (s->training && s->drop_p > 0.f) ? 1 : 0;
  p.salt0 = (int32_t)(l * nm);
  p.drop_p = p.drop ? s->drop_p : 0.f;
  p.seed = s->drop_seed;
  p.ug = s->UG[l];
  p.x = x_res;
  p.ldx = ldx;
  for (int64_t k = 0; k < nm; ++k) {
    const int64_t idx = l * nm + k;
    p.w1[k] = s->w1[idx];
    p.b1[k] = s->b1[idx];
    p.w2[k] = s->w2[idx];
    p.b2[k] = s->b2[idx];
    p.V[k] = s->V[idx];
    p.R[k] = s->R[idx];
    p.A[k] = (k < nm - 1) ? s->A[idx] : nullptr;
    p.M[k] = p.drop ? s->M[idx] : nullptr;
  }
  p.out = out;
  p.ldo = ldo;
  const unsigned blocks = (unsigned)cdiv(s->N, kRows);
  hipLaunchKernelGGL(k_mlp_fwd, dim3(blocks), dim3(mlp_threads(s->D)), mlp_lds_bytes(s->D), st, p);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

int launch_mlp_bwd(const AimxShellStack* s, int64_t l, const float* dy, int64_t lddy, float* const* dV,
                   float* const* dA, float* dug, hipStream_t st) {
  MlpBwd p{};
  const int64_t nm = s->num_mlp;
  p.N = s->N;
  p.D = s->D;
  p.nm = (int32_t)nm;
  p.act = s->act;
  p.drop = (s->training && s->drop_p > 0.f) ? 1 : 0;
  p.drop_p = p.drop ? s->drop_p : 0.f;
  p.dy = dy;
  p.lddy = lddy;
  p.u = s->U[l];
  for (int64_t k = 0; k < nm; ++k) {
    const int64_t idx = l * nm + k;
    p.w1[k] = s->w1[idx];
    p.w2[k] = s->w2[idx];
    p.V[k] = s->V[idx];
    p.M[k] = p.drop ? s->M[idx] : nullptr;
    p.dV[k] = dV[k];
    p.dA[k] = (k < nm - 1) ? dA[k] : nullptr;
  }
  p.dug = dug;
  const unsigned blocks = (unsigned)cdiv(s->N, kRows);
  hipLaunchKernelGGL(k_mlp_bwd, dim3(blocks), dim3(mlp_threads(s->D)), mlp_lds_bytes(s->D), st, p);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

}  // namespace aimx
