// EXPERIMENT — NOT BUILT (not in the Makefile). Kept for the next round's GEMM work.
// Whole-layer fused MLP (2*nm GEMMs with LDS-resident activations and weights). Measured on MI355X
// at c2 (N = 9185, D = 76): 73 us per layer forward vs 44 us for the per-GEMM path it replaces;
// the kernel runs at one wave per SIMD (345 VGPRs) and each of its ~7 serial memory phases costs a
// full load round trip (4-5 us each by s_memtime stamps). Needs: fewer registers (occupancy),
// weights prefetched under the previous GEMM, and larger row tiles before it can win.
// Fused node-update MLP of one shell layer (reference src/models/layers.py:82-106): all of the
// layer's LinearBlock-style MLP blocks in ONE kernel, forward and backward.
//
// Forward, per block k (x_0 = act(u), the first half of [u | g]):
//   v_k = x_k W1_k^T + b1_k ; r_k = dropout(act(v_k)) ; x_{k+1} = r_k W2_k^T + b2_k + x_k
// and the layer output y = x_nm + g (+ the outer residual x, gnn.py:302-306). A workgroup owns 32
// atoms; the block's activations stay in LDS across the 2*nm GEMMs (v_mfma_f32_16x16x4_f32 on
// LDS-resident A and W tiles) and only the tensors the backward needs (V, R, A, dropout masks)
// and the output are written. Backward: the activation-gradient chain of the same blocks,
//   dV_k = (dX W2_k) * mask/(1-p) * act'(V_k) ; dX <- dX + dV_k W1_k ; du = dX * act'(u)
// with dUG = [du | dY] written in place (the weight gradients run later as one grouped launch).
//
// The arithmetic (k order, epilogue operation order) is the unfused path's exactly, so results
// are bit-identical to the per-GEMM path (which remains for D > kMlpMaxD).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 32;        // atoms per workgroup
constexpr int kDP = 80;        // max padded width (D <= 80: c1 38, c2/c3 76)
constexpr int kLS = kDP + 2;   // LDS row stride (bank = 2*row + k for the fragment reads)
constexpr int kMaxBlocks = 8;

struct MlpFwdArgs {
  int64_t N, D;
  int32_t nm, act, drop;
  float drop_p;
  const int64_t* seed;
  int32_t salt0;
  const float* ug;  // [N, 2D]: a0 = act(u) in [0, D), g in [D, 2D)
  int64_t ld_ug;
  const float* x;   // outer residual (nullable)
  int64_t ldx;
  const float* w1[kMaxBlocks];
  const float* b1[kMaxBlocks];
  const float* w2[kMaxBlocks];
  const float* b2[kMaxBlocks];
  float* V[kMaxBlocks];
  float* R[kMaxBlocks];
  float* A[kMaxBlocks];
  uint8_t* M[kMaxBlocks];
  float* out;
  int64_t ldo;
  unsigned long long* stamps;  // diagnostic only (AIMX_MLP_STAMPS): per-workgroup phase cycles
};

struct MlpBwdArgs {
  int64_t N, D;
  int32_t nm, act, drop;
  float drop_p;
  const float* dy;
  int64_t ldy;
  const float* U;
  const float* V[kMaxBlocks];
  const uint8_t* M[kMaxBlocks];
  const float* w1[kMaxBlocks];
  const float* w2[kMaxBlocks];
  float* dV[kMaxBlocks];
  float* dA[kMaxBlocks];  // dA[k]: gradient w.r.t. the output of block k (k < nm - 1)
  float* dUG;             // [N, 2D]
};

// Memory phases issue all of a thread's loads before the first use (clamped, always-valid
// addresses; validity applied by select), so each phase costs one round trip, not one per element.
constexpr int kTilePer = (kBM * kDP + 255) / 256;  // <= 10 elements of a [32 x 80] tile per thread
constexpr int kWPer = (kDP * kDP + 255) / 256;     // <= 25 elements of an [80 x 80] weight per thread

// rows [row0, row0 + rows) x cols [0, D) of a row-major matrix (ld) -> LDS tile (zero padded)
__device__ __forceinline__ void load_tile(const float* __restrict__ g, int64_t ld, int64_t row0, int rows, int D,
                                          int DP, float* T) {
  float v[kTilePer];
  const int tot = kBM * DP;
#pragma unroll
  for (int i = 0; i < kTilePer; ++i) {
    const int e = min((int)threadIdx.x + 256 * i, tot - 1);
    const int m = e / DP, k = e - m * DP;
    v[i] = g[(row0 + min(m, rows - 1)) * ld + min(k, D - 1)];
  }
#pragma unroll
  for (int i = 0; i < kTilePer; ++i) {
    const int e = (int)threadIdx.x + 256 * i;
    if (e < tot) {
      const int m = e / DP, k = e - m * DP;
      T[m * kLS + k] = (m < rows && k < D) ? v[i] : 0.f;
    }
  }
}

// W [D x D] row-major -> LDS image Ws[n][k] = W[n][k] (TRANS: Ws[n][k] = W[k][n]); padding stays 0
template <bool TRANS>
__device__ __forceinline__ void load_weight(const float* __restrict__ W, int D, float* Ws) {
  float v[kWPer];
  const int tot = D * D;
#pragma unroll
  for (int i = 0; i < kWPer; ++i) v[i] = W[min((int)threadIdx.x + 256 * i, tot - 1)];
#pragma unroll
  for (int i = 0; i < kWPer; ++i) {
    const int e = (int)threadIdx.x + 256 * i;
    if (e < tot) {
      const int r = e / D, c = e - r * D;
      if (TRANS)
        Ws[c * kLS + r] = v[i];
      else
        Ws[r * kLS + c] = v[i];
    }
  }
}

// acc[q] += A[m][k] * W[n][k] over k < DP for the wave's tiles t = w + 4q (tile t: mt = t / NT,
// nt = t % NT), q < NV; A and W are LDS images with row stride kLS. NV is a template constant so
// the accumulators update unconditionally (a conditional update makes hipcc copy them out of the
// accumulator registers after every MFMA).
template <int NV, int NT>
__device__ __forceinline__ void mma_tiles_n(const float* As, const float* Ws, int w, int lane, floatx4 (&acc)[3]) {
  constexpr int DP = NT * 16;
  int ao[NV], bo[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int t = w + 4 * q;
    const int mt = t / NT, nt = t - mt * NT;
    ao[q] = (mt * 16 + (lane & 15)) * kLS + (lane >> 4);
    bo[q] = (nt * 16 + (lane & 15)) * kLS + (lane >> 4);
  }
#pragma unroll
  for (int k = 0; k < DP; k += 4) {
#pragma unroll
    for (int q = 0; q < NV; ++q)
      acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(As[ao[q] + k], Ws[bo[q] + k], acc[q], 0, 0, 0);
  }
}

template <int NT>
__device__ __forceinline__ void mma_tiles(const float* As, const float* Ws, int w, int lane, floatx4 (&acc)[3]) {
#pragma unroll
  for (int q = 0; q < 3; ++q) acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nv = (2 * NT - w + 3) / 4;  // tiles w, w+4, w+8 below 2*NT (wave-uniform)
  if (nv >= 3)
    mma_tiles_n<3, NT>(As, Ws, w, lane, acc);
  else if (nv == 2)
    mma_tiles_n<2, NT>(As, Ws, w, lane, acc);
  else if (nv == 1)
    mma_tiles_n<1, NT>(As, Ws, w, lane, acc);
}

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int ACT, int NT>
__global__ __launch_bounds__(256) void k_mlp_fwd(const MlpFwdArgs p) {
  __shared__ float Ws1[kDP * kLS], Ws2[kDP * kLS], As[kBM * kLS], Rs[kBM * kLS], Bs[2][kDP];
  // wave index made provably uniform: the per-wave tile choice is then a scalar branch (a
  // divergent one masks every MFMA and copies its accumulators out after it)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int D = (int)p.D;
  constexpr int DP = NT * 16;
  const int64_t row0 = (int64_t)blockIdx.x * kBM;
  const int rows = (int)min<int64_t>(kBM, p.N - row0);
  for (int e = tid; e < kDP * kLS; e += 256) Ws1[e] = Ws2[e] = 0.f;
  for (int e = tid; e < 2 * kDP; e += 256) Bs[e / kDP][e % kDP] = 0.f;
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t0 = 0, t1 = 0;
  if (p.stamps) t0 = stamp();
  load_tile(p.ug, p.ld_ug, row0, rows, D, DP, As);
  const float scale = p.drop_p < 1.f ? 1.f / (1.f - p.drop_p) : 0.f;
  const uint64_t seed = p.drop ? (uint64_t)*p.seed : 0;
  for (int blk = 0; blk < p.nm; ++blk) {
    __syncthreads();  // previous block's readers of Ws / Bs are done (and the zero fill landed)
    if (p.stamps) { t1 = stamp(); ts[blk == 0 ? 0 : 6] += t1 - t0; t0 = t1; }
    load_weight<false>(p.w1[blk], D, Ws1);
    load_weight<false>(p.w2[blk], D, Ws2);
    if (tid < D) Bs[0][tid] = p.b1[blk][tid];
    else if (tid >= 128 && tid - 128 < D) Bs[1][tid - 128] = p.b2[blk][tid - 128];
    __syncthreads();
    if (p.stamps) { t1 = stamp(); ts[1] += t1 - t0; t0 = t1; }
    floatx4 acc[3];
    mma_tiles<NT>(As, Ws1, w, lane, acc);
    if (p.stamps) { asm volatile("s_nop 0" ::: "memory"); t1 = stamp(); ts[2] += t1 - t0; t0 = t1; }
    const uint32_t salt = (uint32_t)(p.salt0 + blk);
    float* const Vb = p.V[blk];
    float* const Rb = p.R[blk];
    uint8_t* const Mb = p.M[blk];
    float* const Ab = p.A[blk];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = w + 4 * q;
      if (t >= 2 * NT) continue;
      const int mt = t / NT, nt = t - mt * NT;
      const int n = nt * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + (lane >> 4) * 4 + r;
        const bool ok = m < rows && n < D;
        const int64_t gm = row0 + m;
        // epilogue of the unfused linear1: pre = acc + (0 + b1); r = act(pre); dropout
        float add = 0.f;
        add += Bs[0][n];
        float x = acc[q][r] + add;
        if (ok) Vb[gm * D + n] = x;
        x = act_fwd(ACT, x);
        if (p.drop) {
          const bool keep = hash_uniform(seed, salt, (uint64_t)gm * (uint64_t)D + (uint64_t)n) >= p.drop_p;
          x = keep ? x * scale : 0.f;
          if (ok) Mb[gm * D + n] = keep ? 1 : 0;
        }
        x = x * 1.f;
        if (ok) Rb[gm * D + n] = x;
        Rs[m * kLS + n] = ok ? x : 0.f;
      }
    }
    __syncthreads();
    if (p.stamps) { t1 = stamp(); ts[3] += t1 - t0; t0 = t1; }
    mma_tiles<NT>(Rs, Ws2, w, lane, acc);
    if (p.stamps) { t1 = stamp(); ts[4] += t1 - t0; t0 = t1; }
    const bool last = blk == p.nm - 1;
    // the last block's residual terms g and x: all loads issued before use
    float gx[3][4];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) gx[q][r] = 0.f;
    if (last) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int t = min(w + 4 * q, 2 * NT - 1);
        const int mt = t / NT, nt = t - mt * NT;
        const int nn = min(nt * 16 + (lane & 15), D - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = row0 + min(mt * 16 + (lane >> 4) * 4 + r, rows - 1);
          gx[q][r] = p.ug[gm * p.ld_ug + D + nn];
        }
      }
    }
    float xr[3][4];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) xr[q][r] = 0.f;
    if (last && p.x) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int t = min(w + 4 * q, 2 * NT - 1);
        const int mt = t / NT, nt = t - mt * NT;
        const int nn = min(nt * 16 + (lane & 15), D - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t gm = row0 + min(mt * 16 + (lane >> 4) * 4 + r, rows - 1);
          xr[q][r] = p.x[gm * p.ldx + nn];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = w + 4 * q;
      if (t >= 2 * NT) continue;
      const int mt = t / NT, nt = t - mt * NT;
      const int n = nt * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + (lane >> 4) * 4 + r;
        const bool ok = m < rows && n < D;
        const int64_t gm = row0 + m;
        // epilogue of the unfused linear2: add = ((0 + b2) + a) [+ g + x]
        float add = 0.f;
        add += Bs[1][n];
        add += As[m * kLS + n];
        if (last) {
          add += gx[q][r];
          if (p.x) add += xr[q][r];
        }
        const float o = (acc[q][r] + add) * 1.f;
        if (ok) {
          if (last)
            p.out[gm * p.ldo + n] = o;
          else
            Ab[gm * D + n] = o;
        }
        As[m * kLS + n] = ok ? o : 0.f;
      }
    }
  }
  if (p.stamps) {
    const unsigned long long t1e = stamp();
    ts[5] += t1e - t0;
    if (lane == 0)
      for (int k = 0; k < 7; ++k) atomicAdd(&p.stamps[w * 8 + k], ts[k]);
  }

}

template <int ACT, int NT>
__global__ __launch_bounds__(256) void k_mlp_bwd(const MlpBwdArgs p) {
  __shared__ float Wt1[kDP * kLS], Wt2[kDP * kLS], Ds[kBM * kLS], Vs[kBM * kLS];
  // wave index made provably uniform: the per-wave tile choice is then a scalar branch (a
  // divergent one masks every MFMA and copies its accumulators out after it)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int D = (int)p.D;
  constexpr int DP = NT * 16;
  const int64_t row0 = (int64_t)blockIdx.x * kBM;
  const int rows = (int)min<int64_t>(kBM, p.N - row0);
  for (int e = tid; e < kDP * kLS; e += 256) Wt1[e] = Wt2[e] = 0.f;
  load_tile(p.dy, p.ldy, row0, rows, D, DP, Ds);
  __syncthreads();
  for (int e = tid; e < rows * D; e += 256) {  // dg = dY (fused copy into dUG[:, D:])
    const int m = e / D, k = e - m * D;
    p.dUG[(row0 + m) * 2 * D + D + k] = Ds[m * kLS + k];
  }
  const float scale = p.drop_p < 1.f ? 1.f / (1.f - p.drop_p) : 0.f;
  for (int blk = p.nm - 1; blk >= 0; --blk) {
    // C = dX W (no transpose): B[j][n] = W[j][n], kept as Wt[n][j] for the fragment reads
    load_weight<true>(p.w1[blk], D, Wt1);
    load_weight<true>(p.w2[blk], D, Wt2);
    __syncthreads();
    const float* const Vb = p.V[blk];
    const uint8_t* const Mb = p.M[blk];
    float* const dVb = p.dV[blk];
    float* const dAb = blk > 0 ? p.dA[blk - 1] : nullptr;
    floatx4 acc[3];
    mma_tiles<NT>(Ds, Wt2, w, lane, acc);
    // act'(V) and the dropout mask for the wave's elements: all loads first
    float vv[3][4];
    uint8_t mk[3][4];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = min(w + 4 * q, 2 * NT - 1);
      const int mt = t / NT, nt = t - mt * NT;
      const int nn = min(nt * 16 + (lane & 15), D - 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t idx = (row0 + min(mt * 16 + (lane >> 4) * 4 + r, rows - 1)) * D + nn;
        vv[q][r] = Vb[idx];
        mk[q][r] = p.drop ? Mb[idx] : 1;
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = w + 4 * q;
      if (t >= 2 * NT) continue;
      const int mt = t / NT, nt = t - mt * NT;
      const int n = nt * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + (lane >> 4) * 4 + r;
        const bool ok = m < rows && n < D;
        // epilogue of the unfused dV GEMM: (acc + 0) * (act'(V) * mask/(1-p))
        float dg = act_grad(ACT, vv[q][r]);
        if (p.drop) dg *= mk[q][r] ? scale : 0.f;
        const float x = (acc[q][r] + 0.f) * dg;
        if (ok) dVb[(row0 + m) * D + n] = x;
        Vs[m * kLS + n] = ok ? x : 0.f;
      }
    }
    __syncthreads();
    mma_tiles<NT>(Vs, Wt1, w, lane, acc);
    float uu[3][4];
    if (blk == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int t = min(w + 4 * q, 2 * NT - 1);
        const int mt = t / NT, nt = t - mt * NT;
        const int nn = min(nt * 16 + (lane & 15), D - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          uu[q][r] = p.U[(row0 + min(mt * 16 + (lane >> 4) * 4 + r, rows - 1)) * D + nn];
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = w + 4 * q;
      if (t >= 2 * NT) continue;
      const int mt = t / NT, nt = t - mt * NT;
      const int n = nt * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + (lane >> 4) * 4 + r;
        const bool ok = m < rows && n < D;
        const int64_t gm = row0 + m;
        // epilogue of the unfused da_in GEMM: (acc + (0 + da_out)) [* act'(u) for block 0]
        float add = 0.f;
        add += Ds[m * kLS + n];
        float x = acc[q][r] + add;
        if (blk == 0) {
          x = x * act_grad(ACT, uu[q][r]);
          if (ok) p.dUG[gm * 2 * D + n] = x;
        } else {
          x = x * 1.f;
          if (ok) dAb[gm * D + n] = x;
        }
        Ds[m * kLS + n] = ok ? x : 0.f;
      }
    }
    __syncthreads();
  }
}

template <int ACT, int NT, bool FWD>
void* kernel_ptr() {
  if constexpr (FWD)
    return (void*)k_mlp_fwd<ACT, NT>;
  else
    return (void*)k_mlp_bwd<ACT, NT>;
}

template <int ACT, bool FWD>
void* by_nt(int nt) {
  switch (nt) {
    case 1: return kernel_ptr<ACT, 1, FWD>();
    case 2: return kernel_ptr<ACT, 2, FWD>();
    case 3: return kernel_ptr<ACT, 3, FWD>();
    case 4: return kernel_ptr<ACT, 4, FWD>();
    case 5: return kernel_ptr<ACT, 5, FWD>();
    default: return nullptr;
  }
}

// kernel instance for the activation kind and the padded width (NT 16-column tiles)
template <typename F, typename Args, bool FWD>
F pick(int act, int nt) {
  void* k = nullptr;
  switch (act) {
    case ACT_RELU: k = by_nt<ACT_RELU, FWD>(nt); break;
    case ACT_LEAKYRELU: k = by_nt<ACT_LEAKYRELU, FWD>(nt); break;
    case ACT_ELU: k = by_nt<ACT_ELU, FWD>(nt); break;
    case ACT_GELU: k = by_nt<ACT_GELU, FWD>(nt); break;
    case ACT_SILU: k = by_nt<ACT_SILU, FWD>(nt); break;
    case ACT_NONE: k = by_nt<ACT_NONE, FWD>(nt); break;
    default: break;
  }
  return reinterpret_cast<F>(k);
}

}  // namespace

bool mlp_fusable(int64_t D, int64_t nm) {
  static const bool off = getenv("AIMX_NO_FUSED_MLP") != nullptr;  // A/B experiments only
  return !off && D >= 1 && D <= kDP && nm >= 1 && nm <= kMaxBlocks;
}

// Host launchers used by the stack orchestration (stack.hip).
int launch_mlp_fwd(const AimxShellStack* s, int64_t l, const float* x, int64_t ldx, float* out, int64_t ldo,
                   hipStream_t st) {
  MlpFwdArgs p{};
  const int64_t D = s->D, nm = s->num_mlp;
  p.N = s->N;
  p.D = D;
  p.nm = (int32_t)nm;
  p.act = s->act;
  p.drop = (s->training && s->drop_p > 0.f) ? 1 : 0;
  p.drop_p = p.drop ? s->drop_p : 0.f;
  p.seed = p.drop ? s->drop_seed : nullptr;
  p.salt0 = (int32_t)(l * nm);
  p.ug = s->UG[l];
  p.ld_ug = 2 * D;
  p.x = x;
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
  static const bool stamps = getenv("AIMX_MLP_STAMPS") != nullptr;  // diagnostic (never captured)
  static unsigned long long* sbuf = nullptr;
  if (stamps) {
    if (!sbuf) AIMX_CHECK_HIP(hipMalloc(&sbuf, 64 * sizeof(unsigned long long)));
    AIMX_CHECK_HIP(hipMemsetAsync(sbuf, 0, 64 * sizeof(unsigned long long), st));
    p.stamps = sbuf;
  }
  using KF = void (*)(const MlpFwdArgs);
  KF fn = pick<KF, MlpFwdArgs, true>(s->act, (D + 15) / 16);
  if (!fn) return AIMX_EARG;
  hipLaunchKernelGGL(fn, dim3((unsigned)cdiv(s->N, kBM)), dim3(256), 0, st, p);
  AIMX_CHECK_LAUNCH();
  if (stamps) {
    unsigned long long h[64];
    AIMX_CHECK_HIP(hipMemcpyAsync(h, sbuf, sizeof(h), hipMemcpyDeviceToHost, st));
    AIMX_CHECK_HIP(hipStreamSynchronize(st));
    const double nb = (double)cdiv(s->N, kBM);
    fprintf(stderr, "mlp_fwd stamps (avg cycles per workgroup, wave0..3): ");
    const char* names[7] = {"a0", "weights", "gemm1", "epi1", "gemm2", "epi2+end", "epi2(mid)"};
    for (int k = 0; k < 7; ++k) {
      fprintf(stderr, " %s=", names[k]);
      for (int w = 0; w < 4; ++w) fprintf(stderr, "%s%.0f", w ? "/" : "", h[w * 8 + k] / nb);
    }
    fprintf(stderr, "\n");
  }
  return AIMX_OK;
}

int launch_mlp_bwd(const AimxShellStack* s, int64_t l, const float* dy, int64_t ldy, float* const* dV,
                   float* const* dA, float* dUG, hipStream_t st) {
  MlpBwdArgs p{};
  const int64_t D = s->D, nm = s->num_mlp;
  p.N = s->N;
  p.D = D;
  p.nm = (int32_t)nm;
  p.act = s->act;
  p.drop = (s->training && s->drop_p > 0.f) ? 1 : 0;
  p.drop_p = p.drop ? s->drop_p : 0.f;
  p.dy = dy;
  p.ldy = ldy;
  p.U = s->U[l];
  for (int64_t k = 0; k < nm; ++k) {
    const int64_t idx = l * nm + k;
    p.V[k] = s->V[idx];
    p.M[k] = p.drop ? s->M[idx] : nullptr;
    p.w1[k] = s->w1[idx];
    p.w2[k] = s->w2[idx];
    p.dV[k] = dV[k];
    p.dA[k] = (k < nm - 1) ? dA[k] : nullptr;
  }
  p.dUG = dUG;
  using KB = void (*)(const MlpBwdArgs);
  KB fn = pick<KB, MlpBwdArgs, false>(s->act, (D + 15) / 16);
  if (!fn) return AIMX_EARG;
  hipLaunchKernelGGL(fn, dim3((unsigned)cdiv(s->N, kBM)), dim3(256), 0, st, p);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

}  // namespace aimx
