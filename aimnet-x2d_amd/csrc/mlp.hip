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
  int32_t v4;  // fill with 16-byte loads (D, 2D and every weight / row pointer 4-float aligned)
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
  int32_t v4;       // fill with 16-byte loads (D, lddy and every weight / dy pointer 4-float aligned)
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

// ---- Weight-resident variant (small D: every block's weights fit in LDS) --------------------------
// The per-row-tile kernels above re-stream each weight fragment from L2 in every GEMM phase of every
// workgroup, with the first loads of each phase exposed (measured 48 / 54 us per layer at c2 vs
// ~42 / 43 us for the four separate GEMMs). Here a persistent workgroup (one per CU) stages ALL
// 2*nm weight matrices of the layer in LDS once — as k-contiguous rows, transposed for the backward
// — and then walks row chunks of 16*rt atoms: each GEMM phase is rt x CF (16 x 16) output tiles, one
// per wave, over K padded to 16 with zeros, every operand read from LDS by 16-byte ds_reads with the
// k order permuted identically for A and B (lane l supplies k = 16 g + 4 (l >> 4) + j to MFMA step
// j of group g, so one ds_read_b128 per operand feeds 4 v_mfma_f32_16x16x4_f32). Epilogues are the
// per-row-tile kernels' (same dropout hash, salts and rounding order).
constexpr int kWMaxWaves = 16;
constexpr int kMlpwDynLds = 160 * 1024 - 1024;  // + the static pointer table, within one CU's LDS

#ifdef AIMX_MLPW_TRACE  // diagnostics build only: phase timestamps of workgroup 0 (forward)
__device__ long long g_mlpw_trace[64];
#define MLPW_STAMP(k)                                                                           \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x == 0 && (k) < 64) g_mlpw_trace[(k)] = (long long)wall_clock64(); \
  } while (0)
#else
#define MLPW_STAMP(k) \
  do {                \
  } while (0)
#endif

__host__ __device__ inline int pad16(int d) { return (d + 15) / 16 * 16; }
__host__ __device__ inline int wstride(int d) { return pad16(d) + 4; }  // 4 mod 64 or 20 mod 64 ... conflict-free b128

// C tile (t, f) = A[16 t .., :Kp] . Bt[16 f .., :Kp]^T, both LDS images row stride S (k contiguous).
__device__ __forceinline__ floatx4 tile_mma(const float* A, const float* Bt, int S, int Kp, int t, int f) {
  const int lane = threadIdx.x & 63, lr = lane & 15, kq = 4 * (lane >> 4);
  const float* a0 = A + (16 * t + lr) * S + kq;
  const float* b0 = Bt + (16 * f + lr) * S + kq;
  floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int g = 0; g < Kp; g += 16) {
    const floatx4 a = *reinterpret_cast<const floatx4*>(a0 + g);
    const floatx4 b = *reinterpret_cast<const floatx4*>(b0 + g);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
  }
  return acc;
}

// Initial fill of a workgroup's LDS: nmat D x D weights as k-contiguous [Kp][S] images (rows n,
// zero beyond D; TR: transposed, image row n = column n of W, for the backward's B(k, n) = W[k][n])
// and the first row chunk (rows [r0, r0 + R) x cols [0, D) of src, zero beyond D and beyond N).
// Global latency is the cost here (~2 us per dependent round trip on a loaded chip), so every
// thread issues up to kFillU weight loads and kFillR row loads before the first LDS store: one
// round trip for the whole fill at c2's sizes. Matrix pointers come from an LDS table (no private
// arrays, which would live in scratch).
constexpr int kFillW = 8, kFillM = 4, kFillR = 8;

// Workgroup barrier for LDS hand-offs only: the LDS writes are drained (lgkmcnt), outstanding
// global stores are NOT waited for (__syncthreads' fence would wait for every epilogue store).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Buffer descriptor over [p, p + bytes): loads past the extent return 0, so an out-of-range element
// is a load from an address past the end (an ADDRESS select) — a value select after the load lets
// hipcc branch around every load and wait for each one in turn (cdna_hip_programming.md §5 trap (c)).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mlp_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ float mlp_bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

template <bool TR>
__device__ __forceinline__ void fill_lds(float* Wl, const float* const* wtab, int nmat, int D, int Kp, int S,
                                         float* Rl, const float* src, int64_t lds_, int64_t r0, int R, int64_t N) {
  const int NT = blockDim.x, tid = threadIdx.x;
  const int per = Kp * Kp, totr = R * Kp;
  const uint32_t wbytes = 4u * (uint32_t)(D * D), OOB = 0xFFFFFFF0u;
  const int64_t nrows = max<int64_t>(0, min<int64_t>(R, N - r0));
  const __amdgpu_buffer_rsrc_t rr = mlp_rsrc(src + r0 * lds_, (uint32_t)(4 * max<int64_t>(1, nrows * lds_)));
  for (int m0 = 0; m0 < nmat; m0 += kFillM) {
    for (int e0 = 0; e0 < per; e0 += kFillW * NT) {
      float v[kFillM][kFillW], q[kFillR];
#pragma unroll
      for (int mi = 0; mi < kFillM; ++mi) {
        const int m = min(m0 + mi, nmat - 1);
        const __amdgpu_buffer_rsrc_t rw = mlp_rsrc(wtab[m], wbytes);
#pragma unroll
        for (int u = 0; u < kFillW; ++u) {
          const int e = e0 + u * NT + tid, n = e / Kp, k = e - n * Kp;
          const bool ok = e < per && n < D && k < D;
          v[mi][u] = mlp_bload(rw, ok ? 4u * (uint32_t)(TR ? k * D + n : n * D + k) : OOB);
        }
      }
      const bool rows = m0 == 0 && e0 == 0;  // the row chunk rides along with the first batch
#pragma unroll
      for (int u = 0; u < kFillR; ++u) {
        const int e = u * NT + tid, r = e / Kp, c = e - r * Kp;
        const bool ok = rows && e < totr && c < D && r < nrows;
        q[u] = mlp_bload(rr, ok ? 4u * (uint32_t)(r * lds_ + c) : OOB);
      }
#pragma unroll
      for (int mi = 0; mi < kFillM; ++mi) {
        if (m0 + mi >= nmat) break;
#pragma unroll
        for (int u = 0; u < kFillW; ++u) {
          const int e = e0 + u * NT + tid;
          if (e < per) {
            const int n = e / Kp, k = e - n * Kp;
            Wl[(m0 + mi) * Kp * S + n * S + k] = v[mi][u];
          }
        }
      }
      if (rows) {
#pragma unroll
        for (int u = 0; u < kFillR; ++u) {
          const int e = u * NT + tid;
          if (e < totr) {
            const int r = e / Kp, c = e - r * Kp;
            Rl[r * S + c] = q[u];
          }
        }
      }
    }
  }
  for (int e = kFillR * NT + tid; e < totr; e += NT) {  // rows beyond one batch (large R * Kp)
    const int r = e / Kp, c = e - r * Kp;
    Rl[r * S + c] = (c < D && r < nrows) ? src[(r0 + r) * lds_ + c] : 0.f;
  }
}

// fill_lds with 16-byte loads (MlpFwd/MlpBwd.v4: D, the row stride and every pointer 4-float
// aligned). A dword load is address-rate bound at a quarter of a dwordx4's bytes, and the fill's
// ~25 k weight floats per workgroup made it ~7 us of a ~23 us layer at c2. Weights come in as
// float4 along their contiguous dim: [n][k..k+3] stored as one 16-byte LDS write; for TR the
// column run W[k][n..n+3] lands in 4 image rows (4 dword LDS writes). Zero padding as in fill_lds
// (a group is wholly inside D or wholly past it, since D % 4 == 0).
constexpr int kFillW4 = 2, kFillR4 = 2;
template <bool TR>
__device__ __forceinline__ void fill_lds_v4(float* Wl, const float* const* wtab, int nmat, int D, int Kp, int S,
                                            float* Rl, const float* src, int64_t lds_, int64_t r0, int R, int64_t N) {
  const int NT = blockDim.x, tid = threadIdx.x;
  const int kq = Kp / 4, per4 = Kp * kq, totr4 = R * kq;
  const uint32_t wbytes = 4u * (uint32_t)(D * D), OOB = 0xFFFFFFF0u;
  const int64_t nrows = max<int64_t>(0, min<int64_t>(R, N - r0));
  const __amdgpu_buffer_rsrc_t rr = mlp_rsrc(src + r0 * lds_, (uint32_t)(4 * max<int64_t>(1, nrows * lds_)));
  auto ld4 = [](__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  };
  for (int m0 = 0; m0 < nmat; m0 += kFillM) {
    for (int e0 = 0; e0 < per4; e0 += kFillW4 * NT) {
      floatx4 v[kFillM][kFillW4], q[kFillR4];
#pragma unroll
      for (int mi = 0; mi < kFillM; ++mi) {
        const int m = min(m0 + mi, nmat - 1);
        const __amdgpu_buffer_rsrc_t rw = mlp_rsrc(wtab[m], wbytes);
#pragma unroll
        for (int u = 0; u < kFillW4; ++u) {
          // (row a, cols b4..b4+3) of W; TR walks a fastest, so a wave's 4 dword LDS writes per group
          // land on consecutive image columns (conflict-free) instead of rows 4 apart (16-way)
          const int g = e0 + u * NT + tid;
          const int a = TR ? g % Kp : g / kq, b4 = TR ? 4 * (g / Kp) : 4 * (g - a * kq);
          const bool ok = g < per4 && a < D && b4 < D;
          v[mi][u] = ld4(rw, ok ? 4u * (uint32_t)(a * D + b4) : OOB);
        }
      }
      const bool rows = m0 == 0 && e0 == 0;
#pragma unroll
      for (int u = 0; u < kFillR4; ++u) {
        const int g = u * NT + tid, r = g / kq, c = 4 * (g - r * kq);
        const bool ok = rows && g < totr4 && c < D && r < nrows;
        q[u] = ld4(rr, ok ? 4u * (uint32_t)(r * lds_ + c) : OOB);
      }
#pragma unroll
      for (int mi = 0; mi < kFillM; ++mi) {
        if (m0 + mi >= nmat) break;
        float* img = Wl + (m0 + mi) * Kp * S;
#pragma unroll
        for (int u = 0; u < kFillW4; ++u) {
          const int g = e0 + u * NT + tid;
          if (g < per4) {
            const int a = TR ? g % Kp : g / kq, b4 = TR ? 4 * (g / Kp) : 4 * (g - a * kq);
            if (TR) {
#pragma unroll
              for (int j = 0; j < 4; ++j) img[(b4 + j) * S + a] = v[mi][u][j];
            } else {
              *reinterpret_cast<floatx4*>(img + a * S + b4) = v[mi][u];
            }
          }
        }
      }
      if (rows) {
#pragma unroll
        for (int u = 0; u < kFillR4; ++u) {
          const int g = u * NT + tid;
          if (g < totr4) {
            const int r = g / kq, c = 4 * (g - r * kq);
            *reinterpret_cast<floatx4*>(Rl + r * S + c) = q[u];
          }
        }
      }
    }
  }
  for (int g = kFillR4 * NT + tid; g < totr4; g += NT) {  // rows beyond one batch (large R * Kp)
    const int r = g / kq, c = 4 * (g - r * kq);
    *reinterpret_cast<floatx4*>(Rl + r * S + c) =
        ld4(rr, (c < D && r < nrows) ? 4u * (uint32_t)(r * lds_ + c) : OOB);
  }
}

// rows [r0, r0 + R) x cols [0, D) of src (row stride lds_) -> LDS rows of stride S, zero beyond D
// (to Kp) and beyond N
__device__ __forceinline__ void load_rows(float* dst, int S, const float* src, int64_t lds_, int64_t r0, int R, int D,
                                          int Kp, int64_t N) {
  const int total = R * Kp;
  for (int e0 = 0; e0 < total; e0 += kFillR * (int)blockDim.x) {
    float v[kFillR];
#pragma unroll
    for (int u = 0; u < kFillR; ++u) {
      const int e = e0 + u * blockDim.x + threadIdx.x;
      const int r = e / Kp, c = e - r * Kp;
      const bool ok = e < total && c < D && r0 + r < N;
      const float x = src[ok ? (r0 + r) * lds_ + c : 0];
      v[u] = ok ? x : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kFillR; ++u) {
      const int e = e0 + u * blockDim.x + threadIdx.x;
      if (e < total) {
        const int r = e / Kp, c = e - r * Kp;
        dst[r * S + c] = v[u];
      }
    }
  }
}

__global__ __launch_bounds__(64 * kWMaxWaves) void k_mlpw_fwd(const MlpFwd p, int rt) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int D = (int)p.D, Kp = pad16(D), S = wstride(D), CF = Kp / 16, nm = p.nm;
  const int R = 16 * rt;
  float* W = lds;                        // W1_k at 2k, W2_k at 2k+1: [Kp][S] each
  float* Xa = W + 2 * nm * Kp * S;       // block input a_k [R][S]
  float* Hb = Xa + R * S;                // r_k             [R][S]
  float* Bia = Hb + R * S;               // b1_k at 2k, b2_k at 2k+1: [Kp] each
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __shared__ const float* wtab[16];
  __shared__ const float* btab[16];
  if (threadIdx.x < 2 * nm) {
    wtab[threadIdx.x] = (threadIdx.x & 1) ? p.w2[threadIdx.x >> 1] : p.w1[threadIdx.x >> 1];
    btab[threadIdx.x] = (threadIdx.x & 1) ? p.b2[threadIdx.x >> 1] : p.b1[threadIdx.x >> 1];
  }
  for (int e = threadIdx.x; e < R * S; e += blockDim.x) Hb[e] = 0.f;  // k padding of the 2nd GEMM's A
  __syncthreads();
  MLPW_STAMP(0);
  const int64_t N = p.N;
  const int64_t nchunk = (N + R - 1) / R;
  // biases (in flight beside the fill), weights and the first chunk's a0 = act(u) = UG[:, :D] rows
  float bv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = threadIdx.x + u * (int)blockDim.x, m = min(e / Kp, 2 * nm - 1), c = min(e - (e / Kp) * Kp, D - 1);
    bv[u] = btab[m][c];
  }
  if (p.v4)
    fill_lds_v4<false>(W, wtab, 2 * nm, D, Kp, S, Xa, p.ug, 2 * p.D, (int64_t)blockIdx.x * R, R, N);
  else
    fill_lds<false>(W, wtab, 2 * nm, D, Kp, S, Xa, p.ug, 2 * p.D, (int64_t)blockIdx.x * R, R, N);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = threadIdx.x + u * (int)blockDim.x;
    if (e < 2 * nm * Kp) Bia[e] = (e - (e / Kp) * Kp) < D ? bv[u] : 0.f;
  }
  for (int e = threadIdx.x + 2 * (int)blockDim.x; e < 2 * nm * Kp; e += blockDim.x) {  // large nm * Kp
    const int m = e / Kp, c = e - m * Kp;
    Bia[e] = c < D ? btab[m][c] : 0.f;
  }
  lds_sync();
  MLPW_STAMP(1);
  int st = 2;
  (void)st;
  const float scale = drop_scale(p.drop_p);
  const uint64_t seed = p.drop ? (uint64_t)*p.seed : 0;
  const int items = rt * CF;
  const bool single = items <= nw;  // one (tile, fragment) item per wave: prefetch across phases
  for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
    const int64_t r0 = ch * R;
    if (ch != (int64_t)blockIdx.x) {
      __syncthreads();  // the previous chunk's last epilogue reads of Xa are done
      load_rows(Xa, S, p.ug, 2 * p.D, r0, R, D, Kp, N);
      __syncthreads();
    }
    MLPW_STAMP(st++);
    float resid[4] = {0.f, 0.f, 0.f, 0.f};  // the last block's g (+ x), prefetched during its GEMM 1
    for (int k = 0; k < nm; ++k) {
      const bool last = k == nm - 1;
      const float* W1 = W + (2 * k) * Kp * S;
      const float* W2 = W1 + Kp * S;
      float* V = p.V[k];
      float* Rk = p.R[k];
      uint8_t* M = p.M[k];
      const uint32_t salt = (uint32_t)(p.salt0 + k);
      for (int it = wave; it < items; it += nw) {
        const int t = it / CF, f = it - t * CF;
        const int c = 16 * f + (lane & 15), cc = min(c, D - 1);
        if (last && single) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int64_t gc = min(r0 + 16 * t + 4 * (lane >> 4) + i, N - 1);
            resid[i] = p.ug[gc * 2 * p.D + p.D + cc];
            if (p.x) resid[i] += p.x[gc * p.ldx + cc];
          }
        }
        const float bias = Bia[(2 * k) * Kp + cc];
        const floatx4 acc = tile_mma(Xa, W1, S, Kp, t, f);
        if (c < D) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 16 * t + 4 * (lane >> 4) + i;
            const int64_t g = r0 + r;
            const float v = acc[i] + bias;
            float a = act_fwd(p.act, v);
            if (p.drop) {
              const bool keep = hash_uniform(seed, salt, (uint64_t)g * (uint64_t)D + (uint64_t)c) >= p.drop_p;
              a = keep ? a * scale : 0.f;
              if (g < N) M[g * D + c] = keep ? 1 : 0;
            }
            Hb[r * S + c] = a;
            if (g < N) {
              V[g * D + c] = v;
              Rk[g * D + c] = a;
            }
          }
        }
      }
      lds_sync();
      MLPW_STAMP(st++);
      float* Ak = last ? nullptr : p.A[k];
      for (int it = wave; it < items; it += nw) {
        const int t = it / CF, f = it - t * CF;
        const int c = 16 * f + (lane & 15), cc = min(c, D - 1);
        float add[4];
        const float b2 = Bia[(2 * k + 1) * Kp + cc];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          add[i] = b2;
          if (last) {
            if (single) {
              add[i] += resid[i];
            } else {
              const int64_t gc = min(r0 + 16 * t + 4 * (lane >> 4) + i, N - 1);
              float rr = p.ug[gc * 2 * p.D + p.D + cc];
              if (p.x) rr += p.x[gc * p.ldx + cc];
              add[i] += rr;
            }
          }
        }
        const floatx4 acc = tile_mma(Hb, W2, S, Kp, t, f);
        if (c < D) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 16 * t + 4 * (lane >> 4) + i;
            const int64_t g = r0 + r;
            const float a = acc[i] + add[i] + Xa[r * S + c];
            Xa[r * S + c] = a;
            if (g < N) {
              if (last)
                p.out[g * p.ldo + c] = a;
              else
                Ak[g * D + c] = a;
            }
          }
        }
      }
      lds_sync();
      MLPW_STAMP(st++);
    }
  }
  MLPW_STAMP(63);
}

__global__ __launch_bounds__(64 * kWMaxWaves) void k_mlpw_bwd(const MlpBwd p, int rt) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int D = (int)p.D, Kp = pad16(D), S = wstride(D), CF = Kp / 16, nm = p.nm;
  const int R = 16 * rt;
  float* W = lds;                        // W2_k^T at 2k, W1_k^T at 2k+1: [Kp][S] each
  float* DA = W + 2 * nm * Kp * S;       // gradient w.r.t. the current block output [R][S]
  float* DV = DA + R * S;                // dV_k                                     [R][S]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __shared__ const float* wtab[16];
  if (threadIdx.x < 2 * nm) wtab[threadIdx.x] = (threadIdx.x & 1) ? p.w1[threadIdx.x >> 1] : p.w2[threadIdx.x >> 1];
  for (int e = threadIdx.x; e < R * S; e += blockDim.x) DV[e] = 0.f;
  __syncthreads();
  MLPW_STAMP(32);
  int sb = 33;  // backward stamps: slots 32..62 (trace build only)
  (void)sb;
  const int64_t N = p.N;
  const int64_t nchunk = (N + R - 1) / R;
  const float scale = drop_scale(p.drop_p);
  const int items = rt * CF;
  const bool single = items <= nw;  // one (tile, fragment) item per wave: prefetch across phases
  // the dV epilogue operands (act'(v) input and dropout mask) of block k for this wave's item
  float ag[4], mf[4];
  auto pre_dv = [&](int k, int64_t r0, int it) {
    const int t = it / CF, f = it - t * CF, cc = min(16 * f + (lane & 15), D - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t gc = min(r0 + 16 * t + 4 * (lane >> 4) + i, N - 1);
      mf[i] = p.drop ? (p.M[k][gc * D + cc] ? scale : 0.f) : 1.f;
      ag[i] = p.V[k][gc * D + cc];
    }
  };
  if (p.v4)
    fill_lds_v4<true>(W, wtab, 2 * nm, D, Kp, S, DA, p.dy, p.lddy, (int64_t)blockIdx.x * R, R, N);
  else
    fill_lds<true>(W, wtab, 2 * nm, D, Kp, S, DA, p.dy, p.lddy, (int64_t)blockIdx.x * R, R, N);
  // the first dV epilogue's operands, issued AFTER the fill: vmcnt retires in order, so loads issued
  // before it would hold up the fill's LDS writes (these are only needed after the first GEMM)
  if (single && (int64_t)blockIdx.x < nchunk) pre_dv(nm - 1, (int64_t)blockIdx.x * R, wave);
  for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
    const int64_t r0 = ch * R;
    if (ch != (int64_t)blockIdx.x) {
      __syncthreads();
      load_rows(DA, S, p.dy, p.lddy, r0, R, D, Kp, N);
      if (single) pre_dv(nm - 1, r0, wave);
    }
    lds_sync();
    MLPW_STAMP(sb++);
    for (int e = threadIdx.x; e < R * D; e += blockDim.x) {  // dg = dY (from the LDS copy)
      const int r = e / D, c = e - r * D;
      if (r0 + r < N) p.dug[(r0 + r) * 2 * p.D + p.D + c] = DA[r * S + c];
    }
    float uu[4] = {0.f, 0.f, 0.f, 0.f};  // act'(u) input for block 0's dA phase
    for (int k = nm - 1; k >= 0; --k) {
      const float* W2t = W + (2 * k) * Kp * S;
      const float* W1t = W2t + Kp * S;
      float* dVk = p.dV[k];
      for (int it = wave; it < items; it += nw) {  // dV = (dA W2) * mask/(1-p) * act'(v)
        const int t = it / CF, f = it - t * CF;
        const int c = 16 * f + (lane & 15), cc = min(c, D - 1);
        if (!single) pre_dv(k, r0, it);
        if (k == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) uu[i] = p.u[min(r0 + 16 * t + 4 * (lane >> 4) + i, N - 1) * D + cc];
        }
        const floatx4 acc = tile_mma(DA, W2t, S, Kp, t, f);
        if (c < D) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 16 * t + 4 * (lane >> 4) + i;
            const int64_t g = r0 + r;
            const float dv = (g < N) ? acc[i] * mf[i] * act_grad(p.act, ag[i]) : 0.f;
            DV[r * S + c] = dv;
            if (g < N) dVk[g * D + c] = dv;
          }
        }
      }
      lds_sync();
      MLPW_STAMP(sb++);
      float* dAk = k > 0 ? p.dA[k - 1] : nullptr;
      for (int it = wave; it < items; it += nw) {  // dA_k = dA_{k+1} + dV W1 ; k == 0: du = dA_0 act'(u)
        const int t = it / CF, f = it - t * CF;
        const int c = 16 * f + (lane & 15), cc = min(c, D - 1);
        if (single && k > 0) pre_dv(k - 1, r0, it);  // the next block's dV operands
        if (!single && k == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) uu[i] = p.u[min(r0 + 16 * t + 4 * (lane >> 4) + i, N - 1) * D + cc];
        }
        const floatx4 acc = tile_mma(DV, W1t, S, Kp, t, f);
        if (c < D) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 16 * t + 4 * (lane >> 4) + i;
            const int64_t g = r0 + r;
            const float da = DA[r * S + c] + acc[i];
            DA[r * S + c] = da;
            if (g < N) {
              if (k > 0)
                dAk[g * D + c] = da;
              else
                p.dug[g * 2 * p.D + c] = da * act_grad(p.act, uu[i]);
            }
          }
        }
      }
      lds_sync();
      MLPW_STAMP(sb++);
    }
  }
}

#ifdef AIMX_MLPW_TRACE
}  // namespace
extern "C" int aimx_mlpw_trace_read(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mlpw_trace), sizeof(long long) * 64) == hipSuccess ? 0 : -1;
}
namespace {
#endif

size_t mlpw_lds_bytes(int64_t D, int64_t nm, int rt) {
  const int Kp = pad16((int)D), S = wstride((int)D);
  return sizeof(float) * (size_t)((2 * nm * Kp + 2 * 16 * rt) * S + 2 * nm * Kp);  // + the bias table
}

int g_num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

// rows per chunk: enough 16-row tiles that the chunks fit one round of one workgroup per CU, at
// most 4 tiles and 16 waves' worth of (tile, fragment) items, within the LDS
int mlpw_rt(int64_t N, int64_t D, int64_t nm) {
  const int CF = pad16((int)D) / 16;
  const int64_t tiles = (N + 15) / 16;
  int rt = (int)std::min<int64_t>(4, std::max<int64_t>(1, (tiles + g_num_cus() - 1) / g_num_cus()));
  if (const char* e = getenv("AIMX_MLPW_RT")) rt = std::max(1, std::min(4, atoi(e)));  // A/B experiments only
  while (rt > 1 && (rt * CF > 2 * kWMaxWaves || mlpw_lds_bytes(D, nm, rt) > (size_t)kMlpwDynLds)) --rt;
  return rt;
}

bool mlpw_lds_ok(int64_t D, int64_t nm) {
  static const bool set = [] {
    // dynamic LDS cap: the CU's 160 KiB less the kernels' static table (wtab)
    (void)hipFuncSetAttribute((const void*)k_mlpw_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, kMlpwDynLds);
    (void)hipFuncSetAttribute((const void*)k_mlpw_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, kMlpwDynLds);
    return true;
  }();
  (void)set;
  return D >= 1 && D <= 128 && nm >= 1 && nm <= 8 && mlpw_lds_bytes(D, nm, 1) <= (size_t)kMlpwDynLds;
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
// The weight-resident kernels (default for D <= 128 whose weights fit LDS; AIMX_MLPW=0 turns them
// off) or the per-row-tile ones (AIMX_FUSED_MLP=1).
// (read per call, ~6 calls per train step: tests switch the paths inside one process)
bool mlpw_on(int64_t D, int64_t nm) {
  const char* e = getenv("AIMX_MLPW");
  return (!e || atoi(e) != 0) && mlpw_lds_ok(D, nm);
}

bool mlp_fused_ok(int64_t D, int64_t nm) {
  if (mlpw_on(D, nm)) return true;
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
  {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    bool v4 = s->D % 4 == 0 && al(p.ug);
    for (int64_t k = 0; k < nm; ++k) v4 = v4 && al(p.w1[k]) && al(p.w2[k]);
    p.v4 = (v4 && !getenv("AIMX_MLPW_FILL1")) ? 1 : 0;  // AIMX_MLPW_FILL1: dword fill (A/B)
  }
  if (mlpw_on(s->D, nm)) {
    const int rt = mlpw_rt(s->N, s->D, nm);
    const int items = rt * (pad16((int)s->D) / 16);
    const int64_t chunks = cdiv(s->N, 16 * rt);
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(chunks, g_num_cus()));
    hipLaunchKernelGGL(k_mlpw_fwd, dim3(blocks), dim3(64 * std::min(items, kWMaxWaves)), mlpw_lds_bytes(s->D, nm, rt), st,
                       p, rt);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  }
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
  {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    bool v4 = s->D % 4 == 0 && lddy % 4 == 0 && al(dy);
    for (int64_t k = 0; k < nm; ++k) v4 = v4 && al(p.w1[k]) && al(p.w2[k]);
    p.v4 = (v4 && !getenv("AIMX_MLPW_FILL1")) ? 1 : 0;
  }
  if (mlpw_on(s->D, nm)) {
    const int rt = mlpw_rt(s->N, s->D, nm);
    const int items = rt * (pad16((int)s->D) / 16);
    const int64_t chunks = cdiv(s->N, 16 * rt);
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(chunks, g_num_cus()));
    hipLaunchKernelGGL(k_mlpw_bwd, dim3(blocks), dim3(64 * std::min(items, kWMaxWaves)), mlpw_lds_bytes(s->D, nm, rt), st,
                       p, rt);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  }
  const unsigned blocks = (unsigned)cdiv(s->N, kRows);
  hipLaunchKernelGGL(k_mlp_bwd, dim3(blocks), dim3(mlp_threads(s->D)), mlp_lds_bytes(s->D), st, p);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

}  // namespace aimx
