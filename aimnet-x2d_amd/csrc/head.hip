// Fused post-pool head: the per-molecule chain after the graph pool, forward and input-gradient
// backward, each ONE launch.
//
// Reference: GNN.forward, src/models/gnn.py:252-258
//   x = ffn(post_pooling_projection(x_pooled)); s = skip_transform(x); out = output_layer([x | s])
// with ffn = MultiLayerPerceptron (layers.py:222-267) of LinearBlocks (layers.py:170-219):
//   h = dropout(act(y W1^T + b1)); z = h W2^T + b2 (+ y for the middle blocks).
// Every GEMM of the chain has G (molecules, ~520) rows, so launched one by one each is a
// latency-bound ~6-10 us kernel (9 forward + ~15 backward launches at c2, ~280 us per step).
// Here a workgroup of 16 waves owns 16 molecules and runs the whole chain: the activations stay in
// LDS, each wave produces one 16-column fragment per pass and streams its own 16 weight rows
// through a private LDS slice (no workgroup barrier inside a GEMM), every product is
// v_mfma_f32_16x16x4_f32 (exact fp32), and each epilogue (bias, activation with the
// pre-activation saved, hash dropout with its mask, block skip, the [x | s] concat) is applied in
// registers with its global operands loaded before the k loop. The tensors the weight gradients
// need are written to HBM; the weight gradients themselves then run as one grouped launch
// (aimx_wgrad_grouped, K = G). Measured at c2 (MI355X): head forward+backward 284 -> 211 us,
// train step 1190 -> 1094 us.
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kR = 16;          // molecules per workgroup (the MFMA's 16 rows)
constexpr int kBK = 32;         // k slice of the staged weights
constexpr int kP = 4;           // weight slices in flight from global memory
constexpr int kBSt = kBK + 4;   // LDS row stride of a staged slice (16-byte rows; = 36: the
                                //  ds_read_b128 fragment reads of 16 rows hit disjoint banks)
constexpr int kMaxF = 256;      // widest ffn supported (activations [16][2F] stay in LDS)
constexpr int kS1 = kMaxF + 4;      // LDS row stride of the [16][F] activation buffers (= 4 mod 64:
constexpr int kS2 = 2 * kMaxF + 4;  //  conflict-free ds_read_b128 of A) ... of the [16][2F] ones
constexpr int kMaxBlocks = AIMX_HEAD_MAX_BLOCKS;
constexpr int kWaves = 16;              // waves per workgroup: one 16-column fragment each per pass
constexpr int kThreads = 64 * kWaves;   // (a pass covers 256 output columns)
constexpr int kWaveStage = 16 * kBSt;  // floats of one wave's private staged weight slice

// C[16][N] = A[16][K] . B with B(k, n) = Wk[n * ldw + k] (k-contiguous weight rows: the forward's
// nn.Linear weights as they are, the backward's transposed copies); K % 32 == 0; A in LDS (row
// stride lda). Wave w owns output columns n0 + 16 w + [0, 16) of each 256-column pass. The k index
// inside each 16-block is permuted identically for A and B — lane l supplies k = 16 b + 4 (l >> 4)
// + j at MFMA step j — so each lane's A and B operands are one 16-byte ds_read_b128 each.
// `pre(row, col)` returns the epilogue's global operands of one output (float2: bias, the saved
// pre-activation, a mask factor ...); it runs BEFORE the k loop, so those loads land behind the
// MFMA work instead of costing one round trip each afterwards. `epi(row, col, value, pre)` is
// called once per output by the owning thread; a barrier follows the last pass.
template <class Pre, class Epi>
__device__ __forceinline__ void chain_gemm(const float* A, int lda, int K, const float* Wk, int64_t ldw, int N,
                                           float* Bs, Pre pre, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nsl = K / kBK;  // K % 32 == 0 (checked on the host)
  const int lr = lane & 15, lq = 4 * (lane >> 4);
  float* Bw = Bs + wave * kWaveStage;  // this wave's private staging slice [16 rows][kBSt]
  for (int n0 = 0; n0 < N; n0 += 256) {
    // Each wave stages only the 16 weight rows of its own output fragment: full 128-byte row
    // segments from global (lane l: row 8 i + l / 8, k quad l % 8), written to its private LDS
    // slice and read back as MFMA fragments. LDS operations of one wave complete in issue order,
    // so no barrier is needed and the 16 waves run independently (no per-slice skew or sync).
    const float* src[2];
    int dst[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 8 * i + (lane >> 3), kq = (lane & 7) * 4;
      src[i] = Wk + (int64_t)min(n0 + wave * 16 + row, N - 1) * ldw + kq;  // rows past N: dropped
      dst[i] = row * kBSt + kq;
    }
    const int col = n0 + wave * 16 + lr;
    float2 pv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pv[r] = pre((lane >> 4) * 4 + r, min(col, N - 1));
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    floatx4 rg[kP][2];  // register ring: slice s in rg[s % kP]
    auto load = [&](int sl, floatx4 (&r)[2]) {
      const int s = min(sl, nsl - 1);  // unconditional (clamped) loads: no branch-join waits
#pragma unroll
      for (int i = 0; i < 2; ++i) r[i] = *reinterpret_cast<const floatx4*>(src[i] + s * kBK);
    };
#pragma unroll
    for (int q = 0; q < kP; ++q) load(q, rg[q]);
    __builtin_amdgcn_sched_barrier(0);
    const float* a0 = A + lr * lda + lq;
    const float* b0 = Bw + lr * kBSt + lq;
    for (int s0 = 0; s0 < nsl; s0 += kP) {
#pragma unroll
      for (int q = 0; q < kP; ++q) {
        const int sl = s0 + q;
        if (sl < nsl) {  // uniform
#pragma unroll
          for (int i = 0; i < 2; ++i) *reinterpret_cast<floatx4*>(Bw + dst[i]) = rg[q][i];
          load(sl + kP, rg[q]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const floatx4 a = *reinterpret_cast<const floatx4*>(a0 + sl * kBK + 16 * h);
            const floatx4 b = *reinterpret_cast<const floatx4*>(b0 + 16 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
          }
        }
      }
    }
    if (col < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) epi((lane >> 4) * 4 + r, col, acc[r], pv[r]);
    }
  }
  __syncthreads();  // the next GEMM reads what this epilogue wrote / overwrites what this one read
}

// Backward weight operands: the input gradient dY W needs B(k, n) = W[k][n] with k contiguous
// per n, i.e. W^T row-major. One launch writes every head weight's transpose into the workspace,
// K padded to a multiple of 16 with zeros (only the output layer's K = T needs it).
struct TrTable {
  int32_t n;
  const float* src[2 * kMaxBlocks + 4];
  float* dst[2 * kMaxBlocks + 4];
  int32_t rows[2 * kMaxBlocks + 4], cols[2 * kMaxBlocks + 4], ldd[2 * kMaxBlocks + 4];
  int32_t blk0[2 * kMaxBlocks + 5];
};

__global__ __launch_bounds__(256) void k_head_transpose(const TrTable t) {
  __shared__ float tile[32][33];
  int q = 0;
  while (q + 1 < t.n && t.blk0[q + 1] <= (int)blockIdx.x) ++q;
  const int local = blockIdx.x - t.blk0[q];
  const int R = t.rows[q], C = t.cols[q], ldd = t.ldd[q];
  const int tr = local / ((C + 31) / 32), tc = local % ((C + 31) / 32);
  const int r0 = tr * 32, c0 = tc * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < C) ? t.src[q][(int64_t)r * C + c] : 0.f;
  }
  __syncthreads();
  // dst[c][r] = src[r][c]: dst rows = C, row length ldd >= R (zero padded)
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < C && r < ldd) t.dst[q][(int64_t)c * ldd + r] = tile[tx][y];
  }
}

}  // namespace
}  // namespace aimx

using namespace aimx;

namespace aimx {
namespace {

// all LDS is one static array (a workgroup may declare up to 160 KiB on gfx950): 131 KB
constexpr int kHeadLdsFloats = kWaves * kWaveStage + 2 * kR * kS1 + kR * kS2;  // 70 KB

// Backward workspace (floats): transposed weights, K padded to 16: Wo^T [2F][Tp], Ws^T [F][F],
// per block W2^T, W1^T [F][F], Wp^T [H_in][F].
struct HeadWs {
  int64_t wo, ws, w2, w1, wp, total;  // offsets; w2/w1 of block i at w2 + 2 i F^2 / w1 + 2 i F^2
};
__host__ __device__ inline HeadWs head_ws(int64_t F, int64_t Hin, int64_t T, int nb) {
  HeadWs w;
  const int64_t Tp = (T + 31) / 32 * 32;
  w.wo = 0;
  w.ws = 2 * F * Tp;
  w.w2 = w.ws + F * F;
  w.w1 = w.w2 + F * F;
  w.wp = w.ws + F * F + 2 * (int64_t)nb * F * F;
  w.total = w.wp + Hin * F;
  return w;
}

__device__ __forceinline__ float drop_scale(float p) { return p < 1.f ? 1.f / (1.f - p) : 0.f; }

// Forward. LDS: [2 weight stages][3 activation buffers X, H, C] (C = [z | s] of the concat).
__global__ __launch_bounds__(kThreads) void k_head_fwd(const AimxHead h) {
  __shared__ __attribute__((aligned(16))) float lds[kHeadLdsFloats];
  float* Bs = lds;                          // the waves' private staged weight slices
  float* X = lds + kWaves * kWaveStage;     // current block input y (then z)   [16][kS1]
  float* Hb = X + kR * kS1;        // block hidden h                  [16][kS1]
  float* Cb = Hb + kR * kS1;       // x_pooled, then concat [z | s]   [16][kS2]
  const int64_t g0 = (int64_t)blockIdx.x * kR;
  const int F = (int)h.F, Hin = (int)h.H_in, T = (int)h.T;
  const int64_t G = h.G;
  // input rows (x_pooled) -> Cb (as a staging buffer for the first GEMM's A operand)
  for (int e0 = 0; e0 < kR * Hin; e0 += 8 * kThreads) {  // 8 loads in flight per thread
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * kThreads + threadIdx.x, r = e / Hin, c = e - r * Hin;
      const bool ok = e < kR * Hin && g0 + r < G;
      v[u] = h.x0[ok ? (g0 + r) * h.ldx0 + c : 0];
      v[u] = ok ? v[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * kThreads + threadIdx.x, r = e / Hin, c = e - r * Hin;
      if (e < kR * Hin) Cb[r * kS2 + c] = v[u];
    }
  }
  __syncthreads();
  // y0 = x0 Wp^T + bp
  auto bias = [](const float* b) { return [b](int, int c) { return make_float2(b[c], 0.f); }; };
  chain_gemm(Cb, kS2, Hin, h.wp, Hin, F, Bs, bias(h.bp), [&](int r, int c, float v, float2 p) {
    const float y = v + p.x;
    X[r * kS1 + c] = y;
    if (g0 + r < G) h.y0[(g0 + r) * F + c] = y;
  });
  const float scale = drop_scale(h.drop_p);
  const bool drop = h.training && h.drop_p > 0.f && h.seed;
  const uint64_t seed = drop ? (uint64_t)*h.seed : 0;
  for (int i = 0; i < h.nb; ++i) {
    // v = y W1^T + b1 ; h = dropout(act(v))
    float* V = h.v[i];
    float* Hs = h.hid[i];
    uint8_t* M = h.mask[i];
    chain_gemm(X, kS1, F, h.w1[i], F, F, Bs, bias(h.b1[i]), [&](int r, int c, float acc, float2 p) {
      const float v = acc + p.x;
      float a = act_fwd(h.act, v);
      const int64_t g = g0 + r;
      if (drop) {
        const bool keep = hash_uniform(seed, 0x4EADu + (uint32_t)i, (uint64_t)g * (uint64_t)F + (uint64_t)c) >= h.drop_p;
        a = keep ? a * scale : 0.f;
        if (g < G) M[g * F + c] = keep ? 1 : 0;
      }
      Hb[r * kS1 + c] = a;
      if (g < G) {
        V[g * F + c] = v;
        Hs[g * F + c] = a;
      }
    });
    // z = h W2^T + b2 (+ y)
    float* Z = h.z[i];
    const bool skip = h.skip[i] != 0;
    chain_gemm(Hb, kS1, F, h.w2[i], F, F, Bs, bias(h.b2[i]), [&](int r, int c, float acc, float2 p) {
      float z = acc + p.x;
      if (skip) z += X[r * kS1 + c];
      X[r * kS1 + c] = z;
      if (g0 + r < G) Z[(g0 + r) * F + c] = z;
    });
  }
  // s = z Ws^T + bs ; concat [z | s]
  for (int e = threadIdx.x; e < kR * F; e += blockDim.x) {
    const int r = e / F, c = e - r * F;
    Cb[r * kS2 + c] = X[r * kS1 + c];
    if (g0 + r < G) h.cat[(g0 + r) * 2 * F + c] = X[r * kS1 + c];
  }
  // (the copy above finishes before chain_gemm's first barrier; X is only read from here on)
  chain_gemm(X, kS1, F, h.ws, F, F, Bs, bias(h.bs), [&](int r, int c, float acc, float2 p) {
    const float s = acc + p.x;
    Cb[r * kS2 + F + c] = s;
    if (g0 + r < G) h.cat[(g0 + r) * 2 * F + F + c] = s;
  });
  // out = [z | s] Wo^T + bo
  chain_gemm(Cb, kS2, 2 * F, h.wo, 2 * F, T, Bs, bias(h.bo), [&](int r, int c, float acc, float2 p) {
    if (g0 + r < G) h.out[(g0 + r) * h.ldo + c] = acc + p.x;
  });
}

// Input-gradient chain. LDS: [2 weight stages][dZ, dS/dV, dO] activation buffers.
__global__ __launch_bounds__(kThreads) void k_head_bwd(const AimxHead h, const AimxHeadGrad d) {
  __shared__ __attribute__((aligned(16))) float lds[kHeadLdsFloats];
  float* Bs = lds;                          // the waves' private staged weight slices
  float* DZ = lds + kWaves * kWaveStage;    // gradient w.r.t. the current block output  [16][kS1]
  float* DV = DZ + kR * kS1;        // ds, then dv of each block                [16][kS1]
  float* DO = DV + kR * kS1;        // d_out rows                               [16][kS2]
  const int64_t g0 = (int64_t)blockIdx.x * kR;
  const int F = (int)h.F, Hin = (int)h.H_in, T = (int)h.T;
  const int64_t G = h.G;
  const int Tp = (T + 31) / 32 * 32;
  for (int e = threadIdx.x; e < kR * Tp; e += blockDim.x) {
    const int r = e / Tp, c = e - r * Tp;
    DO[r * kS2 + c] = (g0 + r < G && c < T) ? d.d_out[(g0 + r) * d.ld_dout + c] : 0.f;
  }
  __syncthreads();
  const HeadWs L = head_ws(F, Hin, T, h.nb);
  const float* wt = (const float*)d.workspace;
  // d[z | s] = d_out Wo: dz (direct) -> DZ, ds -> DV and HBM (skip_transform's weight gradient)
  auto none = [](int, int) { return make_float2(0.f, 0.f); };
  chain_gemm(DO, kS2, Tp, wt + L.wo, Tp, 2 * F, Bs, none, [&](int r, int c, float v, float2) {
    if (c < F) {
      DZ[r * kS1 + c] = v;
    } else {
      DV[r * kS1 + c - F] = v;
      if (g0 + r < G) d.ds[(g0 + r) * F + c - F] = v;
    }
  });
  // dz += ds Ws
  const int last = h.nb - 1;
  chain_gemm(DV, kS1, F, wt + L.ws, F, F, Bs, none, [&](int r, int c, float v, float2) {
    const float z = DZ[r * kS1 + c] + v;
    DZ[r * kS1 + c] = z;
    if (g0 + r < G) d.dz[last][(g0 + r) * F + c] = z;
  });
  const float scale = drop_scale(h.drop_p);
  const bool drop = h.training && h.drop_p > 0.f && h.seed;
  for (int i = h.nb - 1; i >= 0; --i) {
    // dv = (dz W2) * mask / (1-p) * act'(v)
    const float* V = h.v[i];
    const uint8_t* M = h.mask[i];
    // pre: (act'(v), dropout factor) of the output, loaded before the k loop
    auto dpre = [&](int r, int c) {
      const int64_t g = min(g0 + r, G - 1);
      const float m = drop ? (M[g * F + c] ? scale : 0.f) : 1.f;
      return make_float2(act_grad(h.act, V[g * F + c]), m);
    };
    chain_gemm(DZ, kS1, F, wt + L.w2 + 2 * (int64_t)i * F * F, F, F, Bs, dpre, [&](int r, int c, float acc, float2 p) {
      const int64_t g = g0 + r;
      float dv = 0.f;
      if (g < G) {
        dv = acc * p.y * p.x;
        d.dv[i][g * F + c] = dv;
      }
      DV[r * kS1 + c] = dv;
    });
    // dy = dv W1 (+ dz for a skip block): the gradient w.r.t. this block's input
    const bool skip = h.skip[i] != 0;
    float* dst = i > 0 ? d.dz[i - 1] : d.dy0;
    chain_gemm(DV, kS1, F, wt + L.w1 + 2 * (int64_t)i * F * F, F, F, Bs, none, [&](int r, int c, float acc, float2) {
      float y = acc;
      if (skip) y += DZ[r * kS1 + c];
      DZ[r * kS1 + c] = y;
      if (g0 + r < G) dst[(g0 + r) * F + c] = y;
    });
  }
  // d x_pooled = dy0 Wp
  chain_gemm(DZ, kS1, F, wt + L.wp, F, Hin, Bs, none, [&](int r, int c, float acc, float2) {
    if (g0 + r < G) d.d_x0[(g0 + r) * d.ld_dx0 + c] = acc;
  });
}

bool head_valid(const AimxHead* h) {
  if (!h || h->G < 0 || h->F < 32 || h->F > kMaxF || h->F % 32 || h->H_in < 32 || h->H_in > 2 * kMaxF ||
      h->H_in % 32 || h->T < 1 || h->T > 2 * kMaxF || h->nb < 1 || h->nb > kMaxBlocks)
    return false;
  if (!h->x0 || h->ldx0 < h->H_in || !h->wp || !h->bp || !h->ws || !h->bs || !h->wo || !h->bo || !h->out ||
      h->ldo < h->T || !h->y0 || !h->cat)
    return false;
  for (int i = 0; i < h->nb; ++i)
    if (!h->w1[i] || !h->b1[i] || !h->w2[i] || !h->b2[i] || !h->v[i] || !h->hid[i] || !h->z[i] ||
        (h->training && h->drop_p > 0.f && (!h->mask[i] || !h->seed)))
      return false;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al(h->wp) || !al(h->ws) || !al(h->wo)) return false;
  for (int i = 0; i < h->nb; ++i)
    if (!al(h->w1[i]) || !al(h->w2[i])) return false;
  return true;
}

}  // namespace
}  // namespace aimx

extern "C" int aimx_head_forward(const AimxHead* h, aimx_stream_t stream) {
  if (!head_valid(h)) return AIMX_EARG;
  if (h->G == 0) return AIMX_OK;
  const unsigned blocks = (unsigned)cdiv(h->G, kR);
  hipLaunchKernelGGL(k_head_fwd, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, *h);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" size_t aimx_head_backward_workspace_bytes(const AimxHead* h) {
  if (!head_valid(h)) return 0;
  return sizeof(float) * (size_t)head_ws(h->F, h->H_in, h->T, h->nb).total;
}

extern "C" int aimx_head_backward(const AimxHead* h, const AimxHeadGrad* d, aimx_stream_t stream) {
  if (!head_valid(h) || !d || !d->d_out || d->ld_dout < h->T || !d->d_x0 || d->ld_dx0 < h->H_in || !d->ds ||
      !d->dy0 || !d->workspace || d->workspace_bytes < aimx_head_backward_workspace_bytes(h) ||
      ((uintptr_t)d->workspace & 15))
    return AIMX_EARG;
  for (int i = 0; i < h->nb; ++i)
    if (!d->dz[i] || !d->dv[i]) return AIMX_EARG;
  if (h->G == 0) return AIMX_OK;
  // transposed weight copies (one launch for all of them)
  const HeadWs L = head_ws(h->F, h->H_in, h->T, h->nb);
  float* wt = (float*)d->workspace;
  TrTable t{};
  auto add = [&](const float* src, int R, int C, float* dst, int ldd) {
    const int q = t.n++;
    t.src[q] = src;
    t.dst[q] = dst;
    t.rows[q] = R;
    t.cols[q] = C;
    t.ldd[q] = ldd;
    t.blk0[q + 1] = t.blk0[q] + (int)(cdiv(R, 32) * cdiv(C, 32));
  };
  const int F = (int)h->F, Hin = (int)h->H_in, T = (int)h->T, Tp = (T + 31) / 32 * 32;
  add(h->wo, T, 2 * F, wt + L.wo, Tp);  // Wo [T][2F] -> [2F][Tp]
  add(h->ws, F, F, wt + L.ws, F);
  for (int i = 0; i < h->nb; ++i) {
    add(h->w2[i], F, F, wt + L.w2 + 2 * (int64_t)i * F * F, F);
    add(h->w1[i], F, F, wt + L.w1 + 2 * (int64_t)i * F * F, F);
  }
  add(h->wp, F, Hin, wt + L.wp, F);  // Wp [F][Hin] -> [Hin][F]
  hipLaunchKernelGGL(k_head_transpose, dim3((unsigned)t.blk0[t.n]), dim3(256), 0, (hipStream_t)stream, t);
  AIMX_CHECK_LAUNCH();
  const unsigned blocks = (unsigned)cdiv(h->G, kR);
  hipLaunchKernelGGL(k_head_bwd, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, *h, *d);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
