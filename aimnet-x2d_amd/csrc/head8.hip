// Fused post-pool head on 8-molecule tiles (the default where it applies; head.hip keeps the
// 16-molecule clustered kernels for the other shapes).
//
// Reference: GNN.forward, src/models/gnn.py:252-258
//   x = ffn(post_pooling_projection(x_pooled)); s = skip_transform(x); out = output_layer([x | s])
// ffn = MultiLayerPerceptron (layers.py:222-267) of LinearBlocks (layers.py:170-219):
//   h = dropout(act(y W1^T + b1)); z = h W2^T + b2 (+ y for the middle blocks).
//
// The chain is nine dependent G x F x F GEMMs each way (G ~ 520 molecules), so its time is the
// chain's latency, and a tile's chain runs at the MFMA rate of the CUs it spans. A 16-row tile
// (v_mfma_f32_16x16x4_f32) holds one CU for ~3.4 us per GEMM at F = 256, and splitting it over
// CUs costs an HBM hand-off per GEMM (head.hip's clusters). Here a workgroup owns 8 molecules
// and computes with v_mfma_f32_4x4x1_16b_f32 used as a 4-row x 64-column tile: all 16 blocks take
// the same A (4 rows at one k, broadcast from LDS) and block b the B columns 4b..4b+3, so a lane
// owns one output column and 4 rows (two accumulators: rows 0-3, 4-7). Half the rows per
// workgroup, twice the workgroups, the same MFMA rate: the chain's GEMMs take half as long and no
// inter-workgroup exchange exists.
//
// 16 waves: wave w takes column group w % (F/64) and k range w / (F/64) of every GEMM (F / 64
// groups x 16 / (F / 64) k ranges), so each wave's operand stream is small and 16 streams keep
// enough loads in flight. B(k, n) for 4 consecutive k comes as ONE 16-byte load per lane from a
// k4-interleaved image (k_head8_pack, once per call per direction: the forward's W^T into the
// forward workspace, the backward's W into the backward workspace), held up to 8 items ahead in
// a register ring that runs across GEMM boundaries (the weights do not depend on the
// activations; 4 dword loads per item and a 4-item ring left the stream latency-bound). The k-range
// partial sums meet in LDS and every thread finishes two or four outputs: the fixed-order sum, the
// epilogue (bias, activation with the saved pre-activation, the dropout hash and mask, the block
// skip, the [z | s] concat) and the stores the weight gradients need. The barriers wait on LDS
// only: the global stores stay in flight. The output layer (T outputs, K = 2F) and its backward
// (K = T) are dot products on the vector ALUs.
#include <algorithm>
#include <cstdlib>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) uint8_t gu8;

constexpr int kRows = 8;      // molecules per workgroup (the most: head8_rows)
constexpr int kWaves = 16;    // waves per workgroup
constexpr int kNT = 64 * kWaves;
constexpr int kRingMax = 8;   // B items (4 k each) in flight per wave (fewer when a GEMM has fewer)
// widest F (see head8_ok). 512 (c4) measured slower before the k4-interleaved images and the
// 4-row tiles; with them c4 2.641 -> 2.589 ms (8-row tiles 2.697)
constexpr int kMaxF8 = 512;
constexpr int kMaxGemms = 2 * AIMX_HEAD_MAX_BLOCKS + 2;

__device__ __forceinline__ float drop_scale8(float p) { return p < 1.f ? 1.f / (1.f - p) : 0.f; }

// Workgroup barrier for LDS hand-offs only (global stores are not waited for).
__device__ __forceinline__ void lds_sync8() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Geometry shared by every GEMM of the chain (all are F x F: H_in == F is required).
struct Geo8 {
  int F, cgs, ks, items;  // column groups F/64, k ranges 16/cgs, items (4 k) per wave per GEMM
  int S;                  // LDS row stride of an [8][F] activation tile (== 16 mod 64 floats)
  int S2;                 // ... of the [8][2F] concat tile
};

__host__ __device__ inline Geo8 geo8(int F) {
  Geo8 g;
  g.F = F;
  g.cgs = F / 64;
  g.ks = kWaves / g.cgs;
  g.items = F / (4 * g.ks);
  g.S = (F + 63) / 64 * 64 + 16;
  g.S2 = (2 * F + 63) / 64 * 64 + 16;
  return g;
}

// One wave's operand stream over the chain. GEMM j's B is a k4-interleaved image at tab[j]
// (head8_pack: B(k, n) at ((k / 4) * F + n) * 4 + k % 4), so the wave's 4 k rows of column
// 64 cg + lane are ONE 16-byte load per lane, 1 KiB per wave contiguous. Item s of the stream is
// item s % items of GEMM s / items; past the end it re-reads the last item (never used).
struct BStream8 {
  const gfloat* const* tab;  // per GEMM image base (LDS table of global pointers)
  int n, items, F, k0;       // GEMMs, items per GEMM, row length, first k of the wave's range
  int col;                   // 64 cg + lane
  int j, i;                  // cursor: GEMM, item
  __device__ __forceinline__ void next(floatx4& r) {
    const bool in = j < n;
    const gfloat* b = tab[in ? j : n - 1] + ((int64_t)(k0 / 4 + (in ? i : items - 1)) * F + col) * 4;
    r = *reinterpret_cast<const __attribute__((address_space(1))) floatx4*>(b);
    if (++i == items) {
      i = 0;
      ++j;
    }
  }
};

// This wave's share of one GEMM: rows 0-7 of A (LDS, row stride lda) times its B column group over
// its k range, into acc0 (rows 0-3) / acc1 (rows 4-7) — lane l holds column 64 cg + l.
template <int RW, int RG>
__device__ __forceinline__ void gemm8(const float* A, int lda, int k0, int items, floatx4 (&ring)[RG],
                                      BStream8& bs, floatx4& acc0, floatx4& acc1) {
  const int lane = threadIdx.x & 63;
  const float* a0 = A + (lane & 3) * lda + k0;
  const float* a1 = a0 + 4 * lda;
  acc0 = floatx4{0.f, 0.f, 0.f, 0.f};
  acc1 = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int i0 = 0; i0 < items; i0 += RG) {
#pragma unroll
    for (int q = 0; q < RG; ++q) {
      const int k = 4 * (i0 + q);
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(a0 + k);
      floatx4 x1;
      if (RW == 8) x1 = *reinterpret_cast<const floatx4*>(a1 + k);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(x0[t], ring[q][t], acc0, 0, 0, 0);
        if (RW == 8) acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(x1[t], ring[q][t], acc1, 0, 0, 0);
      }
      bs.next(ring[q]);  // refilled after its last read: the load reuses the registers
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// The wave's partial sums -> red[kq][row][col]
template <int RW>
__device__ __forceinline__ void put_partials(float* red, const Geo8& g, int kq, int col, const floatx4& acc0,
                                             const floatx4& acc1) {
  float* p = red + (int64_t)kq * RW * g.F + col;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    p[r * g.F] = acc0[r];
    if (RW == 8) p[(r + 4) * g.F] = acc1[r];
  }
}

// sum over the k ranges in order
template <int RW>
__device__ __forceinline__ float sum_partials(const float* red, const Geo8& g, int r, int c) {
  float v = red[r * g.F + c];
  for (int q = 1; q < g.ks; ++q) v += red[(int64_t)q * RW * g.F + r * g.F + c];
  return v;
}

struct Lds8 {
  float* X;    // [8][S]  block input y / z (forward); dz (backward)
  float* Hb;   // [8][S]  block hidden h (forward); dv / ds (backward)
  float* Cb;   // [8][S2] x_pooled, then [z | s] (forward); unused (backward)
  float* red;  // [ks][8][F] partial sums
  const gfloat** tab;  // [kMaxGemms] the chain's B operands
};

// + the operand pointer table (kMaxGemms pointers) at the end: every array lives in the dynamic
// region (a static __shared__ ahead of it can shift its base off 16-byte alignment)
__host__ __device__ inline size_t lds8_floats(const Geo8& g, int rw) {
  return (size_t)2 * rw * g.S + (size_t)rw * g.S2 + (size_t)g.ks * rw * g.F + 2 * kMaxGemms;
}

template <int RW>
__device__ __forceinline__ Lds8 carve8(float* lds, const Geo8& g) {
  Lds8 L;
  L.X = lds;
  L.Hb = L.X + RW * g.S;
  L.Cb = L.Hb + RW * g.S;
  L.red = L.Cb + RW * g.S2;
  L.tab = reinterpret_cast<const gfloat**>(L.red + g.ks * RW * g.F);
  return L;
}

// Forward operand table: GEMM order pp, (W1_i, W2_i) for each block, skip; each the row-major
// [F][F] transpose of the nn.Linear weight (B(k, n) = W[n][k]) in the caller's workspace.
template <int RW, int RG>
__global__ __launch_bounds__(kNT) void k_head8_fwd(const AimxHead h, const float* __restrict__ wt) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = (int)h.F, T = (int)h.T, nb = h.nb;
  const Geo8 g = geo8(F);
  const Lds8 L = carve8<RW>(lds, g);
  const gfloat** tab = L.tab;
  const int ng = 2 + 2 * nb;
  if (threadIdx.x < ng) tab[threadIdx.x] = (const gfloat*)(wt + (int64_t)threadIdx.x * F * F);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cg = wave % g.cgs, kq = wave / g.cgs;
  const int64_t G = h.G, g0 = (int64_t)blockIdx.x * RW;
  const float scale = drop_scale8(h.drop_p);
  const bool drop = h.training && h.drop_p > 0.f && h.seed;
  const uint64_t seed = drop ? (uint64_t)*h.seed : 0;
  // x_pooled rows -> Cb[:, :F] (zero past G)
  for (int e = threadIdx.x; e < RW * F; e += kNT) {
    const int r = e / F, c = e - r * F;
    L.Cb[r * g.S2 + c] = (g0 + r < G) ? ((const gfloat*)h.x0)[(g0 + r) * h.ldx0 + c] : 0.f;
  }
  __syncthreads();
  BStream8 bs{tab, ng, g.items, F, kq * 4 * g.items, 64 * cg + lane, 0, 0};
  floatx4 ring[RG];
#pragma unroll
  for (int q = 0; q < RG; ++q) {
    bs.next(ring[q]);
    __builtin_amdgcn_sched_barrier(0);  // in slot order (see mlp.hip mlps_refill)
  }
  floatx4 acc0, acc1;
  const int k0 = kq * 4 * g.items;
  auto gemm = [&](const float* A, int lda) __attribute__((always_inline)) {
    gemm8<RW, RG>(A, lda, k0, g.items, ring, bs, acc0, acc1);
    put_partials<RW>(L.red, g, kq, 64 * cg + lane, acc0, acc1);
    lds_sync8();
  };
  // y0 = x0 Wp^T + bp
  gemm(L.Cb, g.S2);
  for (int e = threadIdx.x; e < RW * F; e += kNT) {
    const int r = e / F, c = e - r * F;
    const float y = sum_partials<RW>(L.red, g, r, c) + ((const gfloat*)h.bp)[c];
    L.X[r * g.S + c] = y;
    if (g0 + r < G) ((gfloat*)h.y0)[(g0 + r) * F + c] = y;
  }
  lds_sync8();
  for (int i = 0; i < nb; ++i) {
    // v = y W1^T + b1 ; h = dropout(act(v))
    gemm(L.X, g.S);
    {
      gfloat* V = (gfloat*)h.v[i];
      gfloat* Hs = (gfloat*)h.hid[i];
      gu8* M = (gu8*)h.mask[i];
      const gfloat* b1 = (const gfloat*)h.b1[i];
      for (int e = threadIdx.x; e < RW * F; e += kNT) {
        const int r = e / F, c = e - r * F;
        const int64_t gr = g0 + r;
        const float v = sum_partials<RW>(L.red, g, r, c) + b1[c];
        float a = act_fwd(h.act, v);
        if (drop) {
          const bool keep = hash_uniform(seed, 0x4EADu + (uint32_t)i, (uint64_t)gr * (uint64_t)F + (uint64_t)c) >= h.drop_p;
          a = keep ? a * scale : 0.f;
          if (gr < G) M[gr * F + c] = keep ? 1 : 0;
        }
        L.Hb[r * g.S + c] = a;
        if (gr < G) {
          V[gr * F + c] = v;
          Hs[gr * F + c] = a;
        }
      }
    }
    lds_sync8();
    // z = h W2^T + b2 (+ y)
    gemm(L.Hb, g.S);
    {
      gfloat* Z = (gfloat*)h.z[i];
      const gfloat* b2 = (const gfloat*)h.b2[i];
      const bool skip = h.skip[i] != 0, last = i == nb - 1;
      for (int e = threadIdx.x; e < RW * F; e += kNT) {
        const int r = e / F, c = e - r * F;
        float z = sum_partials<RW>(L.red, g, r, c) + b2[c];
        if (skip) z += L.X[r * g.S + c];
        L.X[r * g.S + c] = z;
        if (last) L.Cb[r * g.S2 + c] = z;  // the z half of [z | s]
        if (g0 + r < G) {
          Z[(g0 + r) * F + c] = z;
          if (last) ((gfloat*)h.cat)[(g0 + r) * 2 * F + c] = z;
        }
      }
    }
    lds_sync8();
  }
  // s = z Ws^T + bs -> the s half of [z | s]
  gemm(L.X, g.S);
  for (int e = threadIdx.x; e < RW * F; e += kNT) {
    const int r = e / F, c = e - r * F;
    const float s = sum_partials<RW>(L.red, g, r, c) + ((const gfloat*)h.bs)[c];
    L.Cb[r * g.S2 + F + c] = s;
    if (g0 + r < G) ((gfloat*)h.cat)[(g0 + r) * 2 * F + F + c] = s;
  }
  lds_sync8();
  // out = [z | s] Wo^T + bo: one wave per (row, task) dot product of length 2F
  for (int p = wave; p < RW * T; p += kWaves) {
    const int r = p / T, t = p - r * T;
    float acc = 0.f;
    const gfloat* wo = (const gfloat*)h.wo + (int64_t)t * 2 * F;
    for (int k = lane; k < 2 * F; k += 64) acc += L.Cb[r * g.S2 + k] * wo[k];
    acc = wave_sum(acc);
    if (lane == 0 && g0 + r < G) ((gfloat*)h.out)[(g0 + r) * h.ldo + t] = acc + ((const gfloat*)h.bo)[t];
  }
}

// Input-gradient chain. Operands B(k, n) = W[k][n]: the weights themselves (row-major [F][F]),
// GEMM order skip^T, (W2_i^T, W1_i^T) for blocks nb-1 .. 0, pp^T.
template <int RW, int RG>
__global__ __launch_bounds__(kNT) void k_head8_bwd(const AimxHead h, const AimxHeadGrad d, const float* __restrict__ wt) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = (int)h.F, T = (int)h.T, nb = h.nb;
  const Geo8 g = geo8(F);
  const Lds8 L = carve8<RW>(lds, g);
  const gfloat** tab = L.tab;
  const int ng = 2 + 2 * nb;
  if (threadIdx.x < ng) tab[threadIdx.x] = (const gfloat*)(wt + (int64_t)threadIdx.x * F * F);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cg = wave % g.cgs, kq = wave / g.cgs;
  const int64_t G = h.G, g0 = (int64_t)blockIdx.x * RW;
  const float scale = drop_scale8(h.drop_p);
  const bool drop = h.training && h.drop_p > 0.f && h.seed;
  float* DZ = L.X;   // gradient w.r.t. the current block output
  float* DV = L.Hb;  // ds, then dv of each block
  // d[z | s] = d_out Wo (K = T): dz -> DZ, ds -> DV and HBM
  for (int e = threadIdx.x; e < RW * 2 * F; e += kNT) {
    const int r = e / (2 * F), n = e - r * 2 * F;
    float v = 0.f;
    if (g0 + r < G)
      for (int t = 0; t < T; ++t)
        v += ((const gfloat*)d.d_out)[(g0 + r) * d.ld_dout + t] * ((const gfloat*)h.wo)[(int64_t)t * 2 * F + n];
    if (n < F) {
      DZ[r * g.S + n] = v;
    } else {
      DV[r * g.S + n - F] = v;
      if (g0 + r < G) ((gfloat*)d.ds)[(g0 + r) * F + n - F] = v;
    }
  }
  __syncthreads();
  BStream8 bs{tab, ng, g.items, F, kq * 4 * g.items, 64 * cg + lane, 0, 0};
  floatx4 ring[RG];
#pragma unroll
  for (int q = 0; q < RG; ++q) {
    bs.next(ring[q]);
    __builtin_amdgcn_sched_barrier(0);  // in slot order (see mlp.hip mlps_refill)
  }
  floatx4 acc0, acc1;
  const int k0 = kq * 4 * g.items;
  auto gemm = [&](const float* A) __attribute__((always_inline)) {
    gemm8<RW, RG>(A, g.S, k0, g.items, ring, bs, acc0, acc1);
    put_partials<RW>(L.red, g, kq, 64 * cg + lane, acc0, acc1);
    lds_sync8();
  };
  const int last = nb - 1;
  // dz += ds Ws
  gemm(DV);
  for (int e = threadIdx.x; e < RW * F; e += kNT) {
    const int r = e / F, c = e - r * F;
    const float z = DZ[r * g.S + c] + sum_partials<RW>(L.red, g, r, c);
    DZ[r * g.S + c] = z;
    if (g0 + r < G) ((gfloat*)d.dz[last])[(g0 + r) * F + c] = z;
  }
  lds_sync8();
  for (int i = nb - 1; i >= 0; --i) {
    // dv = (dz W2) * mask / (1-p) * act'(v)
    gemm(DZ);
    {
      const gfloat* V = (const gfloat*)h.v[i];
      const gu8* M = (const gu8*)h.mask[i];
      gfloat* DVg = (gfloat*)d.dv[i];
      for (int e = threadIdx.x; e < RW * F; e += kNT) {
        const int r = e / F, c = e - r * F;
        const int64_t gr = g0 + r;
        float dv = 0.f;
        if (gr < G) {
          const float m = drop ? (M[gr * F + c] ? scale : 0.f) : 1.f;
          dv = sum_partials<RW>(L.red, g, r, c) * m * act_grad(h.act, V[gr * F + c]);
          DVg[gr * F + c] = dv;
        }
        DV[r * g.S + c] = dv;
      }
    }
    lds_sync8();
    // dy = dv W1 (+ dz for a skip block): the gradient w.r.t. this block's input
    gemm(DV);
    {
      const bool skip = h.skip[i] != 0;
      gfloat* dst = (gfloat*)(i > 0 ? d.dz[i - 1] : d.dy0);
      for (int e = threadIdx.x; e < RW * F; e += kNT) {
        const int r = e / F, c = e - r * F;
        float y = sum_partials<RW>(L.red, g, r, c);
        if (skip) y += DZ[r * g.S + c];
        DZ[r * g.S + c] = y;
        if (g0 + r < G) dst[(g0 + r) * F + c] = y;
      }
    }
    lds_sync8();
  }
  // d x_pooled = dy0 Wp
  gemm(DZ);
  for (int e = threadIdx.x; e < RW * F; e += kNT) {
    const int r = e / F, c = e - r * F;
    if (g0 + r < G) ((gfloat*)d.d_x0)[(g0 + r) * d.ld_dx0 + c] = sum_partials<RW>(L.red, g, r, c);
  }
}

}  // namespace

// The 8-row kernels apply when every chain GEMM is F x F with F % 64 == 0 and 128 <= F <= kMaxF8
// (H_in == F: the reference's defaults, ffn_hidden_dim = hidden_dim) and the LDS holds the tiles.
bool head8_ok(const AimxHead* h) {
  if (tune_i64("AIMX_HEAD8", 1) == 0) return false;  // test hook: the 16-molecule kernels
  const int64_t F = h->F;
  // the 16 waves split into F / 64 column groups x 16 / (F / 64) k ranges exactly (F = 128, 256,
  // 512). Every workgroup streams all 2 + 2 nb F x F weights through its CU (9.4 MiB at F = 512);
  // F = 512 ran slower than head.hip's clustered kernels until the k4-interleaved images and the
  // 4-row tiles (round 4: c4 2.641 -> 2.589 ms with head8 at F = 512, profiles/r04_ab.txt)
  if (F < 128 || F > kMaxF8 || kWaves % (F / 64) || F % 64 || h->H_in != F || h->nb < 1 || h->nb > AIMX_HEAD_MAX_BLOCKS)
    return false;
  return lds8_floats(geo8((int)F), kRows) * sizeof(float) <= 156 * 1024;
}

size_t head8_forward_workspace_floats(const AimxHead* h) { return (size_t)(2 + 2 * h->nb) * h->F * h->F; }

namespace {
// molecules per workgroup: 4 (one 4-row accumulator per wave) while G / 4 workgroups leave CUs
// idle, 8 (two accumulators, half the weight stream per molecule) once G / 8 alone fills the chip;
// AIMX_HEAD8_ROWS=4|8 forces one (c2, G = 520: 0.7275 ms with 4 vs 0.7678 ms with 8, r4e)
int head8_rows(int64_t G) {
  static const int r = [] {
    return (int)tune_i64("AIMX_HEAD8_ROWS", 0);  // tuning build
  }();
  if (r == 4 || r == 8) return r;
  return G >= 8 * 256 ? 8 : 4;
}

// The chain's B operands as k4-interleaved images (BStream8): forward B(k, n) = W[n][k] (tr), the
// input-gradient chain B(k, n) = W[k][n], in the order each chain reads them. One thread per
// float4 of the image: 4 consecutive k of one column n.
struct Pack8 {
  const float* w[kMaxGemms];
  int32_t n, F, tr;
  floatx4* dst;
};

__global__ __launch_bounds__(256) void k_head8_pack(const Pack8 p) {
  __shared__ const float* tab[kMaxGemms];
  if (threadIdx.x < kMaxGemms) tab[threadIdx.x] = p.w[threadIdx.x];
  __syncthreads();
  const int F = p.F;
  const int64_t per = (int64_t)F * F / 4, total = per * p.n;
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(u / per);
    const int64_t r = u - m * per;
    const int kq = (int)(r / F), nn = (int)(r - (int64_t)kq * F);
    const float* W = tab[m];
    floatx4 v;
    if (p.tr) {
      v = *reinterpret_cast<const floatx4*>(W + (int64_t)nn * F + 4 * kq);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = W[(int64_t)(4 * kq + t) * F + nn];
    }
    p.dst[u] = v;
  }
}

int head8_pack(const AimxHead* h, bool fwd, float* dst, hipStream_t st) {
  Pack8 p{};
  const int nb = h->nb;
  int j = 0;
  if (fwd) {
    p.w[j++] = h->wp;
    for (int i = 0; i < nb; ++i) {
      p.w[j++] = h->w1[i];
      p.w[j++] = h->w2[i];
    }
    p.w[j++] = h->ws;
  } else {
    p.w[j++] = h->ws;
    for (int i = nb - 1; i >= 0; --i) {
      p.w[j++] = h->w2[i];
      p.w[j++] = h->w1[i];
    }
    p.w[j++] = h->wp;
  }
  p.n = j;
  p.F = (int)h->F;
  p.tr = fwd ? 1 : 0;
  p.dst = reinterpret_cast<floatx4*>(dst);
  const int64_t total = (int64_t)p.n * h->F * h->F / 4;
  hipLaunchKernelGGL(k_head8_pack, dim3((unsigned)std::min<int64_t>(cdiv(total, 256), 1024)), dim3(256), 0, st, p);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

template <int RW, int RG>
int head8_launch(const AimxHead* h, const float* wt, const AimxHeadGrad* d, hipStream_t st) {
  static const bool set = [] {
    (void)hipFuncSetAttribute((const void*)k_head8_fwd<RW, RG>, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
    (void)hipFuncSetAttribute((const void*)k_head8_bwd<RW, RG>, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
    return true;
  }();
  (void)set;
  const size_t lds = lds8_floats(geo8((int)h->F), RW) * sizeof(float);
  const unsigned grid = (unsigned)cdiv(h->G, RW);
  if (d)
    hipLaunchKernelGGL((k_head8_bwd<RW, RG>), dim3(grid), dim3(kNT), lds, st, *h, *d, wt);
  else
    hipLaunchKernelGGL((k_head8_fwd<RW, RG>), dim3(grid), dim3(kNT), lds, st, *h, wt);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

// ring depth: kRingMax items, or a GEMM's whole share when it has fewer (F = 128: 4)
template <int RW>
int head8_launch_rg(const AimxHead* h, const float* wt, const AimxHeadGrad* d, hipStream_t st) {
  return geo8((int)h->F).items % kRingMax == 0 ? head8_launch<RW, kRingMax>(h, wt, d, st)
                                                : head8_launch<RW, 4>(h, wt, d, st);
}
}  // namespace

// forward: the chain weights' k4-interleaved images into the workspace, then the chain
int head8_forward(const AimxHead* h, float* wt, hipStream_t st) {
  const int r = head8_pack(h, true, wt, st);
  if (r != AIMX_OK) return r;
  return head8_rows(h->G) == 4 ? head8_launch_rg<4>(h, wt, nullptr, st) : head8_launch_rg<8>(h, wt, nullptr, st);
}

// backward: the images of W itself into the caller's backward workspace (>= head8_forward_workspace_floats)
int head8_backward(const AimxHead* h, const AimxHeadGrad* d, hipStream_t st) {
  float* wt = (float*)d->workspace;
  const int r = head8_pack(h, false, wt, st);
  if (r != AIMX_OK) return r;
  return head8_rows(h->G) == 4 ? head8_launch_rg<4>(h, wt, d, st) : head8_launch_rg<8>(h, wt, d, st);
}

}  // namespace aimx
