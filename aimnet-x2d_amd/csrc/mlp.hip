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
// Launched per GEMM these are 2 * nm kernels per layer and direction, each re-reading its row
// operand from HBM and paying a launch. Two variants keep a row chunk's activations on chip for
// the whole chain:
//   * weight-resident (k_mlpw_*, D <= 128): every block's weights staged in LDS once per CU;
//   * weight-streamed (k_mlps_*, D > 128, where 2 * nm D x D weights exceed the LDS): the weights
//     are pre-packed once per call in MFMA fragment order and each wave streams its own column
//     fragments straight from L2 into a register ring, 4 k-groups ahead, across GEMM boundaries.
// Dropout uses the same hash, salt and index as the per-GEMM path (hash(seed, layer * nm + k,
// row * D + col)), so the masks are identical.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
// global-address-space views of pointers read from LDS tables (a generic pointer makes every access a
// flat op, which the waitcnt pass must treat as both LDS and VMEM: vmcnt(0) lgkmcnt(0) everywhere)
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ float drop_scale(float p) { return p < 1.f ? 1.f / (1.f - p) : 0.f; }

struct MlpFwd {
  int64_t N, D;
  int32_t nm, act, drop, salt0;
  float drop_p;
  const int64_t* seed;
  const float* ug;  // [N, 2D] (row stride ldug): a0 = act(u), g
  int64_t ldug;
  int64_t lda;      // row stride of R and A (V, M: D)
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
  float* dug;       // [N, 2D] (row stride ldug): [du | dY]
  int64_t ldug;
  int64_t lda;      // row stride of dV and dA (V, M, u: D)
  int32_t v4;       // fill with 16-byte loads (D, lddy and every weight / dy pointer 4-float aligned)
};

// ---- Weight-resident variant (small D: every block's weights fit in LDS) --------------------------
// A first per-row-tile chain (16 rows per workgroup, each weight fragment re-streamed from L2 through
// LDS in every GEMM phase, first loads of each phase exposed) measured 48 / 54 us per layer at c2 vs
// ~42 / 43 us for the four separate GEMMs (round 2; removed). Here a persistent workgroup (one per CU) stages ALL
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
  return buffer_rsrc(p, bytes);  // aimx_common.h (the uint32_t halves matter)
}
__device__ __forceinline__ float mlp_bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t off) { return mlp_bload(r, off); }
// buffer stores: an offset past the extent drops the store (rows past N without a branch per element)
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 0);
}
__device__ __forceinline__ void bstore_u8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b8((unsigned char)v, r, off, 0, 0);
}
constexpr uint32_t kDrop = 0xFFFFFFF0u;  // a buffer offset past every extent

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

// columns [D, Kp) of `rows` LDS rows of stride S set to 0
__device__ __forceinline__ void mlps_zero_pad(float* t, int rows, int S, int D, int Kp) {
  const int w = Kp - D;
  for (int e = threadIdx.x; e < rows * w; e += blockDim.x) {
    const int r = e / w;
    t[r * S + D + (e - r * w)] = 0.f;
  }
}

// The weight-streamed kernels' chunk load: rows [r0, r0 + R) x cols [0, D) of src (row stride ld)
// into LDS rows of stride S with every load of a thread in flight at once (one round trip). Thread
// t owns column t mod D of rows t / D, t / D + RG, ... (RG = blockDim.x / D rows per pass: >= 4 for
// one fragment per wave, >= 2 for two, so MAXU = 4 RT NF passes cover R), so its addresses step by a
// uniform stride; rows >= N read 0 through the buffer extent (an address select, not a value select,
// which would wait for each load). The tile's columns D.. are zeroed once per kernel. gdst
// (optional) also receives the values of the rows < N at gdst[(r0 + r) ldg + c].
template <int MAXU>
__device__ __forceinline__ void load_chunk(float* dst, int S, const float* src, int64_t ld, int64_t r0, int R, int D,
                                           int64_t N, float* gdst = nullptr, int64_t ldg = 0) {
  const int RG = (int)blockDim.x / D;
  int rb = (int)threadIdx.x / D, c = (int)threadIdx.x - rb * D;
  // opaque per call: hoisted out of the chunk loop, the MAXU row offsets and conditions would live
  // (spilled) through every GEMM
  asm volatile("" : "+v"(rb), "+v"(c));
  const bool mine = rb < RG;
  const int nrows = (int)max<int64_t>(0, min<int64_t>(R, N - r0));
  const __amdgpu_buffer_rsrc_t rs = mlp_rsrc(src + r0 * ld, (uint32_t)(4 * max<int64_t>(1, (int64_t)nrows * ld)));
  float v[MAXU];
#pragma unroll
  for (int u = 0; u < MAXU; ++u) {
    const int r = rb + u * RG;
    v[u] = mlp_bload(rs, (mine && r < nrows) ? 4u * (uint32_t)(r * ld + c) : 0xFFFFFFF0u);
  }
#pragma unroll
  for (int u = 0; u < MAXU; ++u) {
    const int r = rb + u * RG;
    if (mine && r < R) {
      dst[r * S + c] = v[u];
      if (gdst && r < nrows) gdst[(r0 + r) * ldg + c] = v[u];
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
    fill_lds_v4<false>(W, wtab, 2 * nm, D, Kp, S, Xa, p.ug, p.ldug, (int64_t)blockIdx.x * R, R, N);
  else
    fill_lds<false>(W, wtab, 2 * nm, D, Kp, S, Xa, p.ug, p.ldug, (int64_t)blockIdx.x * R, R, N);
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
      load_rows(Xa, S, p.ug, p.ldug, r0, R, D, Kp, N);
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
            resid[i] = p.ug[gc * p.ldug + p.D + cc];
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
              Rk[g * p.lda + c] = a;
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
              float rr = p.ug[gc * p.ldug + p.D + cc];
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
                Ak[g * p.lda + c] = a;
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
      if (r0 + r < N) p.dug[(r0 + r) * p.ldug + p.D + c] = DA[r * S + c];
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
            if (g < N) dVk[g * p.lda + c] = dv;
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
                dAk[g * p.lda + c] = da;
              else
                p.dug[g * p.ldug + c] = da * act_grad(p.act, uu[i]);
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

// ---- Weight-streamed variant (D > 128) ------------------------------------------------------------
// At c4 / c5 (D = 153 / 307) one block's two D x D weights already exceed the LDS, and per GEMM the
// node update ran as 2 * nm separate MFMA GEMMs of 29-47 us each (16-33 % of the fp32 MFMA peak).
// Here a workgroup owns a chunk of R = 16 rt rows (rt picked so the chunks fill the CUs in one round:
// c4 96 rows, c5 48) and keeps the chain's two activation tiles in LDS (forward: the block input a_k
// and r_k; backward: dA and dV). Wave w owns 16-column fragments w, w + nw, ... (NF of them) of
// every GEMM and all rt row tiles of the chunk, so one B fragment feeds rt MFMAs. The B operand never
// touches LDS: k_mlps_pack lays every weight out once per call in MFMA fragment order (the image of
// matrix m is [fragment f][k group g][lane] float4s: lane l holds B(16 g + 4 (l >> 4) + j, 16 f + (l & 15)),
// j = 0..3, zero outside D x D), so a wave's B for one 16-wide k group is ONE coalesced 1 KiB
// load, streamed from L2 into a register ring P = 4 or 5 groups ahead. The ring runs over the whole chain:
// the next GEMM's first groups are in flight during the current GEMM's last ones and its epilogue.
// The A operand is the k-permuted 16-byte LDS read of the weight-resident kernels (one ds_read_b128
// per row tile feeds 4 MFMAs). Epilogues, dropout hash, salts and outputs (V, R, M, A, out / dV, dA,
// dUG) are the per-GEMM path's.
constexpr int kSMaxThreads = 768;                // <= 12 waves: up to 170 VGPRs per lane
constexpr int kMlpsDynLds = 160 * 1024 - 1024;   // + the static pointer tables

#ifdef AIMX_MLPS_TRACE  // diagnostics build only: per-wave phase timestamps of two workgroups
// [direction][traced workgroup][wave][stamp], written by lane 0 of each wave with a vector store
__device__ long long g_mlps_trace[2][2][12][24];
__device__ __forceinline__ void mlps_stamp(int dir, int k) {
  const int slot = blockIdx.x == 0 ? 0 : blockIdx.x == 77 ? 1 : -1;
  if (slot >= 0 && (threadIdx.x & 63) == 0 && k < 24) {
    const long long t = (long long)wall_clock64();
    __builtin_nontemporal_store(t, &g_mlps_trace[dir][slot][threadIdx.x >> 6][k]);
  }
}
#define MLPS_STAMP(dir, k) mlps_stamp(dir, k)
#else
#define MLPS_STAMP(dir, k) \
  do {                     \
  } while (0)
#endif

struct SGeom {
  int32_t CF;  // 16-wide output fragments of D: pad16(D) / 16
  int32_t G;   // 16-wide k groups streamed per GEMM: CF rounded up to a multiple of the ring depth P
  int32_t S;   // LDS row stride of an activation tile (floats): 16 G + 4 (conflict-free b128 reads)
  int32_t nw;  // waves
};

struct MlpPack {
  const float* w[32];           // layer-major: layer l's matrices at [l * nmat, (l + 1) * nmat)
  int32_t nmat, D, CF, G, tr;  // tr: image of W^T (backward: B(k, n) = W[k][n])
  int32_t nl;                   // layers packed by this launch
  floatx4* dst;                 // the layers' blocks, consecutive: CF * nmat * G * 64 float4s each
};

__global__ void k_mlps_pack(const MlpPack p) {
  // images of one layer: [f][phase][g][lane] (BStream); p.nmat = 2 nm phases of one layer
  const int64_t per = (int64_t)p.CF * p.nmat * p.G * 64, total = per * p.nl;
  __shared__ const float* tab[32];
  if (threadIdx.x < 32) tab[threadIdx.x] = p.w[threadIdx.x];
  __syncthreads();
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = u / per, uv = u - l * per;
    const int lane = (int)(uv & 63);
    const int64_t q = uv >> 6;
    const int g = (int)(q % p.G);
    const int m = (int)((q / p.G) % p.nmat);
    const int f = (int)(q / ((int64_t)p.G * p.nmat));
    const int n = 16 * f + (lane & 15), k0 = 16 * g + 4 * (lane >> 4);
    const float* W = tab[l * p.nmat + m];
    floatx4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + j;
      v[j] = (n < p.D && k < p.D) ? (p.tr ? W[k * p.D + n] : W[n * p.D + k]) : 0.f;
    }
    p.dst[u] = v;
  }
}

// One k group of the chain's GEMM stream: acc[t][i] += A(rows of tile t, k group g) . B(k group, fragment i).
// Row tiles go in pairs (two independent accumulators per B value), each pair's A operands read just
// before its MFMAs: all RT tiles' A reads in flight at once would hold 4 RT VGPRs.
template <int RT, int NF, int NA = NF>  // NA: the wave's active fragments (0 .. NA-1 of NF)
__device__ __forceinline__ void mlps_group(floatx4 (&acc)[RT][NF], const float* As, int S, int g, const floatx4 (&b)[NF]) {
  const int lane = threadIdx.x & 63, lr = lane & 15, lq = 4 * (lane >> 4);
  const float* a0 = As + lr * S + 16 * g + lq;
#pragma unroll
  for (int t0 = 0; t0 < RT; t0 += 2) {
    constexpr int kW = 2;
    floatx4 a[kW];
#pragma unroll
    for (int u = 0; u < kW; ++u)
      if (t0 + u < RT) a[u] = *reinterpret_cast<const floatx4*>(a0 + 16 * (t0 + u) * S);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < kW; ++u)
#pragma unroll
        for (int i = 0; i < NA; ++i)
          if (t0 + u < RT) acc[t0 + u][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][j], b[i][j], acc[t0 + u][i], 0, 0, 0);
    if (t0 + 2 < RT) __builtin_amdgcn_sched_barrier(0);
  }
}

// The B stream of one wave: items s = (phase, k group) in chain order. An image block holds, per
// fragment f, all 2 nm phases' G k groups back to back ([f][phase][g][lane] float4s; G >= CF,
// G % P == 0, groups past CF zero), so item s of fragment f is ONE pointer step from item s - 1, and
// item s always sits in ring slot s % P (every GEMM starts at slot 0).
template <int NF>
struct BStream {
  const floatx4* ptr[NF];  // this lane's float4 of the next item, per fragment
  const floatx4* last[NF];  // the last item (loads past the end re-read it: never used)
  __device__ __forceinline__ void next(floatx4 (&r)[NF]) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      r[i] = *ptr[i];
      ptr[i] = ptr[i] + 64 < last[i] ? ptr[i] + 64 : last[i];
    }
  }
  __device__ __forceinline__ void init(const floatx4* img, const int (&fr)[NF], int total) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      ptr[i] = img + (int64_t)fr[i] * total * 64 + lane;
      last[i] = ptr[i] + (int64_t)(total - 1) * 64;
    }
  }
};

// The k group loop of one GEMM of the chain (G groups from ring slot 0), keeping the ring P ahead
// inside the GEMM. The last P groups load nothing: the next GEMM's first P items are loaded by the
// caller after this GEMM's epilogue (mlps_refill), so that at every wait for a ring slot the only
// newer vector-memory operations are ring loads. (With the refills crossing into the next GEMM,
// the epilogue's ~3 x 4 RT NF global stores came after them; vmcnt counts stores too, the
// counter's range was exceeded, and hipcc waited for vmcnt(0) at every loop head: at c4 / c5 the
// whole ring drained every P groups.)
// full: every fragment of the wave is real; else its last one lies past CF and its MFMAs are skipped
// (a wave-uniform branch per k group; fragment counts per SIMD are balanced by the plan, mlps_plan)
template <int RT, int NF>
__device__ __forceinline__ void mlps_group_any(floatx4 (&acc)[RT][NF], const float* As, int S, int g,
                                               const floatx4 (&b)[NF], bool full) {
  if (NF == 1 || full)
    mlps_group<RT, NF, NF>(acc, As, S, g, b);
  else
    mlps_group<RT, NF, (NF > 1 ? NF - 1 : 1)>(acc, As, S, g, b);
}

template <int RT, int NF, int P>
__device__ __forceinline__ void mlps_gemm(floatx4 (&acc)[RT][NF], floatx4 (&ring)[P][NF], BStream<NF>& bs, const float* As,
                                          int S, int G, bool full) {
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int i = 0; i < NF; ++i) acc[t][i] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int g0 = 0; g0 < G - P; g0 += P) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      mlps_group_any<RT, NF>(acc, As, S, g0 + q, ring[q], full);
      // refill the slot only after its MFMAs have read it: the load then targets the same registers
      // (a refill issued before the last read needs fresh registers and a copy at the loop's back
      // edge, and copying a register with a load in flight waits for that load)
      bs.next(ring[q]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int q = 0; q < P; ++q) {
    mlps_group_any<RT, NF>(acc, As, S, G - P + q, ring[q], full);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The next GEMM's first P items (clamped re-reads of the last item after the chain's end), issued
// after an epilogue's global stores (see mlps_gemm).
// The loads are pinned in slot order: hipcc would otherwise schedule them freely, and where a
// GEMM is entered from two paths whose slots were filled in different orders (the preload and a
// refill) it can only wait for all of them (vmcnt(0)) before the first MFMA.
template <int NF, int P>
__device__ __forceinline__ void mlps_refill(floatx4 (&ring)[P][NF], BStream<NF>& bs) {
#pragma unroll
  for (int q = 0; q < P; ++q) {
    bs.next(ring[q]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// p.X[k] for a uniform runtime k without indexing the kernel-argument array (dynamic indexing copies
// the whole argument struct to scratch): scalar loads at fixed offsets and selects
template <class T>
__device__ __forceinline__ T pick8(T const (&a)[8], int k) {
  T r = a[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) r = (k == i) ? a[i] : r;
  return r;
}

template <int RT, int NF, int P>
__global__ __launch_bounds__(kSMaxThreads) void k_mlps_fwd(const MlpFwd p, const floatx4* __restrict__ img, const SGeom geo) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  MLPS_STAMP(0, 0);
  constexpr int R = 16 * RT;
  // epilogue operands prefetched into registers during the GEMM where they fit (else loaded in the
  // epilogue): 8 RT NF VGPRs
  const int D = (int)p.D, CF = geo.CF, G = geo.G, S = geo.S, nw = geo.nw, nm = p.nm;
  float* Xa = lds;              // block input a_k [R][S]
  float* Hb = lds + R * S;      // r_k             [R][S]
  float* Bia = lds + 2 * R * S;  // b1_k at 2k, b2_k at 2k+1: [16 CF] each
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 15;
  for (int e = threadIdx.x; e < 2 * nm * 16 * CF; e += blockDim.x) {
    const int m = e / (16 * CF), c = e - m * (16 * CF);
    const float* bb = pick8((m & 1) ? p.b2 : p.b1, m >> 1);
    Bia[e] = c < D ? bb[c] : 0.f;
  }
  const int64_t N = p.N, nchunk = cdiv(N, R);
  const int nph = 2 * nm;
  int fr[NF];
  bool fok[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    fok[i] = wave + i * nw < CF && 16 * (wave + i * nw) + lr < D;
    fr[i] = min(wave + i * nw, CF - 1);
  }
  // all NF fragments real (wave-uniform: readfirstlane)
  const bool full = __builtin_amdgcn_readfirstlane(wave + (NF - 1) * nw) < CF;
  const float scale = drop_scale(p.drop_p);
  const uint64_t seed = p.drop ? (uint64_t)*p.seed : 0;
  // the last block's residual operands as buffer loads (an absent x reads 0: no branch per load)
  const __amdgpu_buffer_rsrc_t rug = mlp_rsrc(p.ug, (uint32_t)(4 * N * p.ldug));
  const __amdgpu_buffer_rsrc_t rx_ = mlp_rsrc(p.x, p.x ? (uint32_t)(4 * ((N - 1) * p.ldx + D)) : 0u);
  // k padding (columns D .. 16 G) of both tiles: the chunk loads and the epilogues write columns < D only
  mlps_zero_pad(Xa, 2 * R, S, D, 16 * G);
  MLPS_STAMP(0, 1);
  for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
    const int64_t r0c = ch * R;
    __syncthreads();  // the previous chunk's last reads of Xa are done
    load_chunk<4 * RT * NF>(Xa, S, p.ug, p.ldug, r0c, R, D, N);  // a0 = act(u) = UG[:, :D]; zero beyond N
    __syncthreads();
    MLPS_STAMP(0, 2);
    BStream<NF> bs;
    bs.init(img, fr, nph * G);
    floatx4 ring[P][NF];
    mlps_refill<NF, P>(ring, bs);
    floatx4 acc[RT][NF];
    for (int ph = 0; ph < nph; ++ph) {
      // an opaque per-GEMM copy of the chunk origin: every epilogue address derives from it, so the
      // compiler recomputes them per GEMM instead of hoisting RT x NF x 4 of them out of the loop
      int64_t r0 = r0c;
      asm volatile("" : "+s"(r0));
      const int k = ph >> 1;
      const bool w1 = (ph & 1) == 0, last = ph == nph - 1;
      float bia[NF];
#pragma unroll
      for (int i = 0; i < NF; ++i) bia[i] = Bia[ph * 16 * CF + 16 * fr[i] + lr];
      mlps_gemm<RT, NF, P>(acc, ring, bs, w1 ? Xa : Hb, S, G, full);
      MLPS_STAMP(0, 3 + 3 * ph);
      // everything the epilogue addresses derives from these opaque copies, so none of it is
      // computed ahead of the GEMM and held across it
      int lo = lane;
      asm volatile("" : "+s"(r0), "+v"(lo));
      const int lr = lo & 15, lq = 4 * (lo >> 4);
      const uint32_t nd = (uint32_t)(N * D);
      if (w1) {  // v = a W1^T + b1 ; r = dropout(act(v))
        const __amdgpu_buffer_rsrc_t rV = mlp_rsrc(pick8(p.V, k), 4u * nd);
        const __amdgpu_buffer_rsrc_t rR = mlp_rsrc(pick8(p.R, k), 4u * (uint32_t)(N * p.lda));
        const __amdgpu_buffer_rsrc_t rM = mlp_rsrc(pick8(p.M, k), p.drop ? nd : 0u);
        const uint32_t salt = (uint32_t)(p.salt0 + k);
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int i = 0; i < NF; ++i) {
            if (!fok[i]) continue;
            const int c = 16 * fr[i] + lr;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * t + lq + r;
              const int64_t gr = r0 + row;
              const uint32_t o = (uint32_t)gr * (uint32_t)D + (uint32_t)c;
              const bool in = gr < N;
              const float v = acc[t][i][r] + bia[i];
              float a = act_fwd(p.act, v);
              if (p.drop) {
                const bool keep = hash_uniform(seed, salt, (uint64_t)o) >= p.drop_p;
                a = keep ? a * scale : 0.f;
                bstore_u8(rM, in ? o : kDrop, keep ? 1u : 0u);
              }
              Hb[row * S + c] = a;
              bstore(rV, in ? 4u * o : kDrop, v);
              bstore(rR, in ? 4u * ((uint32_t)gr * (uint32_t)p.lda + (uint32_t)c) : kDrop, a);
            }
          }
      } else {  // a_{k+1} = r W2^T + b2 + a_k (+ g + x after the last block)
        const uint32_t ldo = last ? (uint32_t)p.ldo : (uint32_t)p.lda;
        const __amdgpu_buffer_rsrc_t rO = last ? mlp_rsrc(p.out, 4u * (uint32_t)((N - 1) * p.ldo + D))
                                               : mlp_rsrc(pick8(p.A, k), 4u * (uint32_t)(N * p.lda));
        // the last block's residual operands g and x, a fragment's loads all issued before their
        // first use (one round trip per fragment). Loaded during the GEMM instead, they slowed its k
        // loop by more (queued ahead of the weight ring's loads, or stalling the MFMAs' issue in a
        // burst: c4 +4-5 us); all fragments at once held too many registers for NF = 2
#pragma unroll
        for (int i = 0; i < NF; ++i) {
          float rg[RT][4], rx[RT][4];
          if (last) {
            const int c = min(16 * fr[i] + lr, D - 1);
#pragma unroll
            for (int t = 0; t < RT; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const uint32_t gq = (uint32_t)min(r0 + 16 * t + lq + r, N - 1);
                rg[t][r] = bload(rug, 4u * (gq * (uint32_t)p.ldug + (uint32_t)(D + c)));
                rx[t][r] = bload(rx_, 4u * (gq * (uint32_t)p.ldx + (uint32_t)c));  // 0 without x
              }
          }
          if (!fok[i]) continue;
          const int c = 16 * fr[i] + lr;
#pragma unroll
          for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * t + lq + r;
              const int64_t gr = r0 + row;
              float a = (acc[t][i][r] + bia[i]) + Xa[row * S + c];
              if (last) a = (a + rg[t][r]) + rx[t][r];
              Xa[row * S + c] = a;
              bstore(rO, gr < N ? 4u * ((uint32_t)gr * ldo + (uint32_t)c) : kDrop, a);
            }
        }
      }
      MLPS_STAMP(0, 4 + 3 * ph);
      mlps_refill<NF, P>(ring, bs);
      lds_sync();  // hand the tile to the next GEMM
      MLPS_STAMP(0, 5 + 3 * ph);
    }
  }
}

template <int RT, int NF, int P>
__global__ __launch_bounds__(kSMaxThreads) void k_mlps_bwd(const MlpBwd p, const floatx4* __restrict__ img, const SGeom geo) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  MLPS_STAMP(1, 0);
  constexpr int R = 16 * RT;
  const int D = (int)p.D, CF = geo.CF, G = geo.G, S = geo.S, nw = geo.nw, nm = p.nm;
  float* DA = lds;          // gradient w.r.t. the current block output [R][S]
  float* DV = lds + R * S;  // dV_k                                     [R][S]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 15;
  const int64_t N = p.N, nchunk = cdiv(N, R);
  const int nph = 2 * nm;
  int fr[NF];
  bool fok[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    fok[i] = wave + i * nw < CF && 16 * (wave + i * nw) + lr < D;
    fr[i] = min(wave + i * nw, CF - 1);
  }
  // all NF fragments real (wave-uniform: readfirstlane)
  const bool full = __builtin_amdgcn_readfirstlane(wave + (NF - 1) * nw) < CF;
  const float scale = drop_scale(p.drop_p);
  mlps_zero_pad(DA, 2 * R, S, D, 16 * G);  // k padding of DA and DV
  MLPS_STAMP(1, 1);
  for (int64_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
    const int64_t r0c = ch * R;
    __syncthreads();
    load_chunk<4 * RT * NF>(DA, S, p.dy, p.lddy, r0c, R, D, N, p.dug + p.D, p.ldug);  // and dg = dY
    __syncthreads();
    MLPS_STAMP(1, 2);
    BStream<NF> bs;
    bs.init(img, fr, nph * G);
    floatx4 ring[P][NF];
    mlps_refill<NF, P>(ring, bs);
    floatx4 acc[RT][NF];
    for (int ph = 0; ph < nph; ++ph) {
      int64_t r0 = r0c;  // opaque per GEMM (see k_mlps_fwd)
      asm volatile("" : "+s"(r0));
      const int k = nm - 1 - (ph >> 1);
      const bool dv = (ph & 1) == 0;
      mlps_gemm<RT, NF, P>(acc, ring, bs, dv ? DA : DV, S, G, full);
      MLPS_STAMP(1, 3 + 3 * ph);
      int lo = lane;  // opaque copies: see k_mlps_fwd
      asm volatile("" : "+s"(r0), "+v"(lo));
      const int lr = lo & 15, lq = 4 * (lo >> 4);
      // per fragment: the epilogue's operands (dV: v and the dropout mask; dA of block 0: u), every
      // load issued before the first use (one round trip per fragment, see k_mlps_fwd), then its
      // outputs
      const uint32_t ldd = dv ? (uint32_t)p.lda : k > 0 ? (uint32_t)p.lda : (uint32_t)p.ldug;
      const __amdgpu_buffer_rsrc_t rout = dv      ? mlp_rsrc(pick8(p.dV, k), 4u * (uint32_t)(N * p.lda))
                                          : k > 0 ? mlp_rsrc(pick8(p.dA, k - 1), 4u * (uint32_t)(N * p.lda))
                                                  : mlp_rsrc(p.dug, 4u * (uint32_t)(N * p.ldug));
      const gfloat* V = (const gfloat*)(dv ? pick8(p.V, k) : p.u);
      const gu8* M = (dv && p.drop) ? (const gu8*)pick8(p.M, k) : (const gu8*)V;
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        float ev[RT][4];
        uint32_t em[RT][4];
        if (dv || k == 0) {
          const uint32_t c = (uint32_t)min(16 * fr[i] + lr, D - 1);
#pragma unroll
          for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint32_t o = (uint32_t)min(r0 + 16 * t + lq + r, N - 1) * (uint32_t)D + c;
              ev[t][r] = V[o];
              em[t][r] = (uint32_t)M[o];  // used only with dropout (else a byte of V: ignored)
            }
        }
        if (!fok[i]) continue;
        const int c = 16 * fr[i] + lr;
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * t + lq + r;
            const int64_t gr = r0 + row;
            float o;
            if (dv) {  // dV = (dA W2) * mask/(1-p) * act'(v)
              const float m = p.drop ? (em[t][r] ? scale : 0.f) : 1.f;
              o = (gr < N) ? acc[t][i][r] * m * act_grad(p.act, ev[t][r]) : 0.f;
              DV[row * S + c] = o;
            } else {  // dA_k = dA_{k+1} + dV W1 ; k == 0: du = dA_0 act'(u) -> dUG[:, :D]
              const float da = DA[row * S + c] + acc[t][i][r];
              DA[row * S + c] = da;
              o = k == 0 ? da * act_grad(p.act, ev[t][r]) : da;
            }
            bstore(rout, gr < N ? 4u * ((uint32_t)gr * ldd + (uint32_t)c) : kDrop, o);
          }
      }
      MLPS_STAMP(1, 4 + 3 * ph);
      mlps_refill<NF, P>(ring, bs);
      lds_sync();
      MLPS_STAMP(1, 5 + 3 * ph);
    }
  }
}

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
  if (const int64_t f = tune_i64("AIMX_MLPW_RT", 0)) rt = (int)std::max<int64_t>(1, std::min<int64_t>(4, f));  // tuning build only
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

// ---- weight-streamed geometry and launches ----
struct MlpsPlan {
  bool ok;
  int RT, NF, P;
  SGeom geo;
  unsigned blocks;
  size_t lds;
};

MlpsPlan mlps_plan(int64_t N, int64_t D) {
  MlpsPlan pl{};
  const int CF = (int)cdiv(D, 16);
  if (D < 1 || CF > 24) return pl;  // beyond 2 fragments per wave: the per-GEMM path
  // waves and fragments per wave: wave w owns fragments w, w + nw, ...; the SIMD running waves
  // s, s + 4, ... carries the sum of their fragment counts. One fragment per wave up to 12; above,
  // two per wave with as many waves (<= 12) as leave the busiest SIMD the fewest fragments (c5's
  // 20: 12 waves, 8 of two fragments and 4 of one -> 5 per SIMD, where 10 waves of two put 6 on two
  // SIMDs and 4 on the others); a wave whose second fragment lies past CF skips its MFMAs
  auto busiest = [&](int nw) {
    int m = 0;
    for (int sd = 0; sd < 4; ++sd) {
      int f = 0;
      for (int w = sd; w < nw; w += 4) f += (int)cdiv(std::max(CF - w, 0), nw);
      m = std::max(m, f);
    }
    return m;
  };
  int nw = CF;
  if (CF > 12) {
    int best = 1 << 30;
    for (int cand = (int)cdiv(CF, 2); cand <= kSMaxThreads / 64; ++cand)
      if (busiest(cand) < best) best = busiest(cand), nw = cand;
  }
  pl.NF = (int)cdiv(CF, nw);
  pl.geo.CF = CF;
  // ring depth P in {5, 4}: the k groups per GEMM rounded up to a multiple of it (fewer zero groups
  // first, then the deeper ring)
  const int g5 = (int)cdiv(CF, 5) * 5, g4 = (int)cdiv(CF, 4) * 4;
  pl.P = g5 <= g4 ? 5 : 4;
  pl.geo.G = std::min(g5, g4);
  pl.geo.S = 16 * pl.geo.G + 4;
  pl.geo.nw = nw;
  // (two workgroups per CU, 5 waves per SIMD at <= 96 VGPRs, measured no faster at c4: 2.894 vs
  // 2.888 ms — 430 chunks of 3 row tiles leave the CUs holding two the busiest — and removed)
  const int rt_max = pl.NF == 1 ? 7 : 3;
  // enough rows per chunk that the chunks fit one round of one workgroup per CU
  const int64_t slots = g_num_cus();
  int rt = (int)std::min<int64_t>(rt_max, std::max<int64_t>(1, cdiv(cdiv(std::max<int64_t>(N, 1), slots), 16)));
  if (const int64_t f = opt_i64("AIMX_MLPS_RT", 0)) rt = (int)std::max<int64_t>(1, std::min<int64_t>(rt_max, f));  // test hook
  // two activation tiles + the forward's bias table (2 nm x 16 CF floats, nm <= 8), per workgroup
  auto lds = [&](int r) { return sizeof(float) * (size_t)(2 * 16 * r * pl.geo.S + 2 * 8 * 16 * CF); };
  const size_t cap = (size_t)kMlpsDynLds;
  while (rt > 1 && lds(rt) > cap) --rt;
  if (lds(rt) > cap) return pl;
  pl.RT = rt;
  pl.lds = lds(rt);
  pl.blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(N, 16 * rt), slots));
  pl.ok = true;
  return pl;
}

template <int RT, int NF, int P>
int mlps_launch(const MlpsPlan& pl, const MlpFwd* pf, const MlpBwd* pb, const float* img, hipStream_t st) {
  static const bool set = [] {
    (void)hipFuncSetAttribute((const void*)k_mlps_fwd<RT, NF, P>, hipFuncAttributeMaxDynamicSharedMemorySize, kMlpsDynLds);
    (void)hipFuncSetAttribute((const void*)k_mlps_bwd<RT, NF, P>, hipFuncAttributeMaxDynamicSharedMemorySize, kMlpsDynLds);
    return true;
  }();
  (void)set;
  const dim3 grid(pl.blocks), block(64 * pl.geo.nw);
  if (pf)
    hipLaunchKernelGGL((k_mlps_fwd<RT, NF, P>), grid, block, pl.lds, st, *pf, reinterpret_cast<const floatx4*>(img),
                       pl.geo);
  else
    hipLaunchKernelGGL((k_mlps_bwd<RT, NF, P>), grid, block, pl.lds, st, *pb, reinterpret_cast<const floatx4*>(img),
                       pl.geo);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

int mlps_dispatch(const MlpsPlan& pl, const MlpFwd* pf, const MlpBwd* pb, const float* img, hipStream_t st) {
#define AIMX_MLPS_CASE(rt, nf)                                                          \
  if (pl.RT == rt && pl.NF == nf)                                                       \
    return pl.P == 5 ? mlps_launch<rt, nf, 5>(pl, pf, pb, img, st) : mlps_launch<rt, nf, 4>(pl, pf, pb, img, st);
  AIMX_MLPS_CASE(1, 1) AIMX_MLPS_CASE(2, 1) AIMX_MLPS_CASE(3, 1) AIMX_MLPS_CASE(4, 1) AIMX_MLPS_CASE(5, 1)
  AIMX_MLPS_CASE(6, 1) AIMX_MLPS_CASE(7, 1) AIMX_MLPS_CASE(1, 2) AIMX_MLPS_CASE(2, 2) AIMX_MLPS_CASE(3, 2)
#undef AIMX_MLPS_CASE
  return AIMX_EARG;
}

// floats of one packed weight image: CF fragments x G k groups x 256
int64_t mlps_image_floats(int64_t D) {
  const MlpsPlan pl = mlps_plan(1, D);
  return (int64_t)pl.geo.CF * pl.geo.G * 256;
}

}  // namespace

// The weight-resident kernels: default for D <= 128 whose weights fit the LDS (the test hook
// AIMX_MLPW = 0 turns them off: the per-GEMM path's parity tests). Read per call.
bool mlpw_on(int64_t D, int64_t nm) { return opt_i64("AIMX_MLPW", 1) != 0 && mlpw_lds_ok(D, nm); }

// The weight-streamed kernels: everything the weight-resident ones do not take, in fp32 (AMP keeps
// the per-GEMM path's bf16 operands), up to D = 384 and 8 blocks. Test hook AIMX_MLPS: 0 turns them off
// (the per-GEMM path), 1 makes them take small D too.
bool mlps_on(int64_t N, int64_t D, int64_t nm, int32_t precision) {
  const int64_t mode = opt_i64("AIMX_MLPS", -1);
  if (mode == 0 || precision == AIMX_PREC_BF16 || nm < 1 || nm > 8) return false;
  if (mode != 1 && mlpw_on(D, nm)) return false;
  return mlps_plan(N, D).ok;
}

// The fused kernels address their row operands through raw buffer descriptors (buffer_rsrc): 32-bit
// byte extents, kBufDrop past them. `ld` is the widest row stride of any operand of the call (the
// stack's [x | F] rows, its output and upstream-gradient rows); larger batches take the per-GEMM path.
static bool mlp_extent_ok(int64_t N, int64_t D, int64_t ld) {
  return 4 * (std::max<int64_t>(N, 1) * std::max<int64_t>(ld, 2 * D) + 2 * D) < (int64_t)kBufDrop - 64;
}

bool mlp_fused_ok(int64_t N, int64_t D, int64_t nm, int32_t precision, int64_t ld) {
  if (!mlp_extent_ok(N, D, ld)) return false;
  if (opt_i64("AIMX_MLPS", -1) == 1) return mlps_on(N, D, nm, precision);
  return mlpw_on(D, nm) || mlps_on(N, D, nm, precision);
}

size_t mlp_pack_floats(const AimxShellStack* s) {
  if (!mlps_on(s->N, s->D, s->num_mlp, s->precision) ||
      !mlp_extent_ok(s->N, s->D, std::max({stack_ld_f(s), stack_ld_ug(s), stack_ld_act(s), s->out_ld})))
    return 0;
  return (size_t)(s->num_layers * 2 * s->num_mlp * mlps_image_floats(s->D));
}

// Every layer's MLP weights as MFMA-fragment images (k_mlps_pack), in the order the chain reads
// them: forward W1_0, W2_0, W1_1, ... per layer; backward (transposed) W2_{nm-1}, W1_{nm-1}, ..., W1_0.
// As many layers per launch as their 2 nm matrices fit the 32-entry table (c4 / c5: all 3 layers in
// one launch instead of one per layer: 3 x 4.7 us -> one).
int launch_mlp_pack(const AimxShellStack* s, bool bwd, float* dst, hipStream_t st) {
  const int64_t nm = s->num_mlp, L = s->num_layers, D = s->D;
  const MlpsPlan pl = mlps_plan(1, D);
  const int64_t per = 2 * nm * mlps_image_floats(D) / 4;  // float4s per layer block
  const int64_t lpl = std::max<int64_t>(1, 32 / (2 * nm));  // layers per launch
  for (int64_t l0 = 0; l0 < L; l0 += lpl) {
    const int64_t nl = std::min(lpl, L - l0);
    MlpPack p{};
    p.nmat = (int32_t)(2 * nm);
    for (int64_t l = l0; l < l0 + nl; ++l)
      for (int64_t j = 0; j < 2 * nm; ++j) {
        const int64_t k = bwd ? nm - 1 - (j >> 1) : (j >> 1);
        const bool w2 = bwd ? (j & 1) == 0 : (j & 1) == 1;
        p.w[(l - l0) * 2 * nm + j] = w2 ? s->w2[l * nm + k] : s->w1[l * nm + k];
      }
    p.D = (int32_t)D;
    p.CF = pl.geo.CF;
    p.G = pl.geo.G;
    p.tr = bwd ? 1 : 0;
    p.nl = (int32_t)nl;
    p.dst = reinterpret_cast<floatx4*>(dst) + l0 * per;
    const int64_t blocks = std::min<int64_t>(cdiv(per * nl, 256), 4096);
    hipLaunchKernelGGL(k_mlps_pack, dim3((unsigned)blocks), dim3(256), 0, st, p);
    AIMX_CHECK_LAUNCH();
  }
  return AIMX_OK;
}

int launch_mlp_fwd(const AimxShellStack* s, int64_t l, const float* x_res, int64_t ldx, float* out, int64_t ldo,
                   const float* pack, hipStream_t st) {
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
  p.ldug = stack_ld_ug(s);
  p.lda = stack_ld_act(s);
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
    bool v4 = s->D % 4 == 0 && p.ldug % 4 == 0 && al(p.ug);
    for (int64_t k = 0; k < nm; ++k) v4 = v4 && al(p.w1[k]) && al(p.w2[k]);
    p.v4 = v4 ? 1 : 0;
  }
  if (!pack && mlpw_on(s->D, nm)) {
    const int rt = mlpw_rt(s->N, s->D, nm);
    const int items = rt * (pad16((int)s->D) / 16);
    const int64_t chunks = cdiv(s->N, 16 * rt);
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(chunks, g_num_cus()));
    hipLaunchKernelGGL(k_mlpw_fwd, dim3(blocks), dim3(64 * std::min(items, kWMaxWaves)), mlpw_lds_bytes(s->D, nm, rt), st,
                       p, rt);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  }
  if (!pack) return AIMX_EARG;
  return mlps_dispatch(mlps_plan(s->N, s->D), &p, nullptr, pack + l * 2 * nm * mlps_image_floats(s->D), st);
}

int launch_mlp_bwd(const AimxShellStack* s, int64_t l, const float* dy, int64_t lddy, float* const* dV,
                   float* const* dA, float* dug, const float* pack, hipStream_t st) {
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
  p.ldug = stack_ld_ug(s);
  p.lda = stack_ld_act(s);
  {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    bool v4 = s->D % 4 == 0 && lddy % 4 == 0 && al(dy);
    for (int64_t k = 0; k < nm; ++k) v4 = v4 && al(p.w1[k]) && al(p.w2[k]);
    p.v4 = v4 ? 1 : 0;
  }
  if (!pack && mlpw_on(s->D, nm)) {
    const int rt = mlpw_rt(s->N, s->D, nm);
    const int items = rt * (pad16((int)s->D) / 16);
    const int64_t chunks = cdiv(s->N, 16 * rt);
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(chunks, g_num_cus()));
    hipLaunchKernelGGL(k_mlpw_bwd, dim3(blocks), dim3(64 * std::min(items, kWMaxWaves)), mlpw_lds_bytes(s->D, nm, rt), st,
                       p, rt);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  }
  if (!pack) return AIMX_EARG;
  return mlps_dispatch(mlps_plan(s->N, s->D), nullptr, &p, pack + l * 2 * nm * mlps_image_floats(s->D), st);
}

}  // namespace aimx

#ifdef AIMX_MLPS_TRACE
extern "C" int aimx_mlps_trace_read(long long* out) {  // 2 x 2 x 12 x 24 stamps (wall clock, 100 MHz)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(aimx::g_mlps_trace), sizeof(long long) * 2 * 2 * 12 * 24) == hipSuccess
             ? 0
             : -1;
}
#endif
