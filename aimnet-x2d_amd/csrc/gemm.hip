// Fused fp32 GEMM on CDNA4 matrix cores for the node-update MLP and the dense projections.
//
// Reference: ShellConvolutionLayer.forward, src/models/layers.py:82-106 (nn.Linear = addmm,
// SiLU, Dropout, residual adds), the projections in gnn.py:224-258 and their autograd backward.
// Every contraction is fp32, so the MFMA is v_mfma_f32_16x16x4_f32: exact f32 products
// accumulated as a k-ordered fmaf chain at the f32 matrix rate (~157 TF/s chip); gfx950 has no
// xf32 path.
//
// Shapes on this path are small and latency-bound (M = atoms ~1e4, N, K = 38..2150), so the
// design goal is few dependent round trips per block and enough blocks per CU:
//  * 256 threads = 4 waves in a 2x2 grid over a BM x BN tile (64x64, 64x32 or 32x32, chosen so the
//    grid covers the chip), each wave (BM/2) x (BN/2) as 16x16 accumulators;
//  * K advances in 64-deep slices; the next slice's global loads are issued into registers before
//    the 16 MFMA k-steps of the current slice run from LDS (one exposed round trip per 64 of K);
//  * the LDS image follows the coalesced direction of each operand: k-contiguous operands
//    (row-major X, W of Y = X W^T) are stored row-major with a 66-float row stride (the two k
//    columns a 32-lane group reads fall on disjoint banks: bank = 2*row + k), m/n-contiguous
//    operands (dY^T of the weight gradient) are stored k-major with a (BM+16)-float stride;
//  * long-K / small-MN products (weight gradients, K = atoms) split K across workgroups; the
//    partial slabs are reduced IN the launch by the last-arriving workgroup of each tile
//    (sc1 slab stores/loads + a self-resetting agent-scope arrival counter, MI355X_MICROARCH.md
//    §visibility "Valid forms"), in slab order: deterministic, no atomics on the data, no extra
//    launch.
// Epilogue (fused, see include/aimx.h): bias, residuals, pre-activation store, activation,
// hash-dropout with mask store, mask/act' multiplication for the backward, and an implicit ones
// column that turns a weight-gradient GEMM's last column into the bias gradient.
#include <algorithm>
#include <cstring>
#include <cstdlib>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kBK = 32;

// Epilogue over the NE outputs a thread owns, in two phases. epi_load issues every global load
// the epilogue needs (C for beta, bias, residuals, act' pre-activation, dropout mask) and folds
// them into two values per element (the additive term and the gradient factor); it depends only
// on the element coordinates, so a kernel may run it BEFORE its main loop and let the loads land
// behind the MFMA work. epi_apply then needs only the accumulators and does the stores.
template <int NE>
struct EpiPre {
  float add[NE];
  float dg[NE];
};

template <int NE>
__device__ __forceinline__ void epi_load(const AimxGemmArgs& a, const int (&m)[NE], const int (&n)[NE],
                                         EpiPre<NE>& p) {
  // Every load below is unconditional from a clamped address (selects, not branches), and every
  // optional operand is tested once outside its element loop, so all NE elements' loads are in
  // flight together.
  int64_t mc[NE];
  int nc[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const bool ones = (a.ones_col != 0) & (n[e] == a.N - 1);
    const bool in = (m[e] < a.M) & (n[e] < a.N) & !ones;
    mc[e] = in ? m[e] : 0;
    nc[e] = in ? n[e] : 0;
  }
#pragma unroll
  for (int e = 0; e < NE; ++e) p.add[e] = 0.f;
  if (a.beta != 0.f) {
#pragma unroll
    for (int e = 0; e < NE; ++e) p.add[e] += a.beta * a.C[mc[e] * a.ldc + nc[e]];
  }
  if (a.bias) {
#pragma unroll
    for (int e = 0; e < NE; ++e) p.add[e] += a.bias[nc[e]];
  }
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    if (a.res[r]) {
      const float* __restrict__ rp = a.res[r];
      const int64_t ld = a.ldres[r];
#pragma unroll
      for (int e = 0; e < NE; ++e) p.add[e] += rp[mc[e] * ld + nc[e]];
    }
  }
  if (a.dact_pre) {
#pragma unroll
    for (int e = 0; e < NE; ++e) p.dg[e] = act_grad(a.dact_kind, a.dact_pre[mc[e] * a.lddact + nc[e]]);
  } else {
#pragma unroll
    for (int e = 0; e < NE; ++e) p.dg[e] = 1.f;
  }
  const float scale = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
  if (a.mask_in) {
#pragma unroll
    for (int e = 0; e < NE; ++e) p.dg[e] *= a.mask_in[mc[e] * a.ldmask + nc[e]] ? scale : 0.f;
  }
}

template <int NE>
__device__ __forceinline__ void epi_apply(const AimxGemmArgs& a, const int (&m)[NE], const int (&n)[NE],
                                          const float (&v)[NE], const EpiPre<NE>& p) {
  bool ok[NE], ones[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    ones[e] = (a.ones_col != 0) & (n[e] == a.N - 1);
    ok[e] = (m[e] < a.M) & (n[e] < a.N);
  }
  const float scale = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
  float x[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) x[e] = v[e] + p.add[e];
  if (a.act_ncols > 0) {
    if (a.pre) {
#pragma unroll
      for (int e = 0; e < NE; ++e)
        if (ok[e] & !ones[e] & (n[e] < a.act_ncols)) a.pre[m[e] * a.ldpre + n[e]] = x[e];
    }
    if (a.act >= 0) {
#pragma unroll
      for (int e = 0; e < NE; ++e)
        if (n[e] < a.act_ncols) x[e] = act_fwd(a.act, x[e]);
    }
  }
  if (a.mask_out) {
    const uint64_t seed = (uint64_t)*a.drop_seed;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const bool keep =
          hash_uniform(seed, a.drop_salt, (uint64_t)(m[e] + a.m_base) * (uint64_t)a.N + (uint64_t)n[e]) >= a.drop_p;
      x[e] = keep ? x[e] * scale : 0.f;
      if (ok[e] & !ones[e]) a.mask_out[m[e] * a.ldmask + n[e]] = keep ? 1 : 0;
    }
  }
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    if (!ok[e]) continue;
    if (ones[e])
      a.col_out[m[e]] = v[e];
    else
      a.C[m[e] * a.ldc + n[e]] = x[e] * p.dg[e];
  }
}

template <int NE>
__device__ __forceinline__ void epilogue_n(const AimxGemmArgs& a, const int (&m)[NE], const int (&n)[NE],
                                           float (&v)[NE]) {
  EpiPre<NE> p;
  epi_load<NE>(a, m, n, p);
  epi_apply<NE>(a, m, n, v, p);
}

// Buffer descriptor over [p, p + bytes): out-of-range loads return 0 (used as the M/N/K edge
// padding), 32-bit byte offsets (fewer VGPRs than 64-bit flat addresses). Inputs are made
// provably wave-uniform with readfirstlane so hipcc does not waterfall the loads (guide T8/T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return buffer_rsrc(p, bytes);  // aimx_common.h (the uint32_t halves matter)
}

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  // the b32 builtin returns the raw bits as an integer: reinterpret, never convert
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// Split-K slab hand-off between workgroups without fences (MI355X_MICROARCH.md "Valid forms",
// row 1): every slab byte is stored and loaded with 16-byte `sc1` (device-coherent) buffer
// accesses; each storing wave drains (vmcnt 0) before the workgroup barrier, one lane then adds
// to the tile's agent-scope counter, and the workgroup whose add returns S-1 reduces. An agent
// release per workgroup (an XCD-wide L2 write-back, serialised per XCD) cost ~0.7 us per block.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSC1 = 16;  // buffer cache-policy bit 4 = sc1
__device__ __forceinline__ void store_sc1(__amdgpu_buffer_rsrc_t r, uint32_t voff, floatx4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, 0, kSC1);
}
__device__ __forceinline__ floatx4 load_sc1(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, kSC1));
}

// AK: A is k-contiguous (sak == 1) -> row-major LDS image (row stride BK+2: bank = 2*row + k,
// conflict-free for the 16x16x4 fragment reads); else A is m-contiguous (sam == 1) -> k-major
// image (stride BM+16). BKC: the same for B with n in place of m.
__device__ __forceinline__ floatx4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Extent of the non-empty hop chunks (AimxGemmArgs.zc_*): E = width * (1 + c), c = 1 + the last
// chunk holding an edge. The row pointers are wave-uniform, so these are a handful of scalar loads.
__device__ __forceinline__ int zc_extent(const int32_t* rp, int64_t rows, int chunks, int64_t width) {
  int c = 0;
  for (int j = 0; j < chunks; ++j)
    if (rp[(int64_t)(j + 1) * rows] > rp[(int64_t)j * rows]) c = j + 1;
  return (int)(width * (1 + c));
}

// Plain zero store of one BM x BN output tile (zc_dim 1: a tile wholly inside the empty chunks).
template <int BM, int BN>
__device__ __forceinline__ void zero_tile(const AimxGemmArgs& a, int m0, int n0, int M, int Nreal) {
  for (int e = threadIdx.x; e < BM * BN; e += 256) {
    const int m = m0 + e / BN, n = n0 + e % BN;
    if (m < M && n < Nreal) a.C[(int64_t)m * a.ldc + n] = 0.f;
  }
}

// V4: both operands staged with 16-byte buffer loads (one dwordx4 moves 1 KiB per wave; dword
// loads are address-rate bound at a quarter of that). Requires the contiguous extent of each
// operand to be a multiple of 4 floats and 16-byte aligned rows (checked by the host), so a float4
// is wholly valid or wholly outside: invalid ones are pointed past the descriptor's extent and
// read as zeros (an address select — no value select for hipcc to turn into a branch).
// BF (AimxGemmArgs.precision == AIMX_PREC_BF16, the AMP path): operands are rounded to bf16 (RNE)
// as they are staged into LDS, always as a k-contiguous [m][k] / [n][k] image (row stride BK + 8
// bf16 = 80 B: the 16-byte fragment reads of a 16-lane group hit disjoint banks), and each 32-deep
// slice is ONE v_mfma_f32_16x16x32_bf16 per fragment pair (fp32 accumulation, fp32 epilogue).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int BM, int BN, bool AK, bool BKC, bool V4, bool BF>
__global__ __launch_bounds__(256) void k_gemm(const AimxGemmArgs a, int kchunk, uint32_t a_bytes, uint32_t b_bytes) {
  constexpr int BK = kBK;
  constexpr int SH = BK + 8;                       // BF: bf16 row stride of both LDS images
  constexpr int LAH = BM * SH, LBH = BN * SH;      // BF: bf16 elements per stage and operand
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int SA = AK ? BK + 2 : BM + 16;
  constexpr int SB = BKC ? BK + 2 : BN + 16;
  constexpr int LA = AK ? BM * SA : BK * SA;
  constexpr int LB = BKC ? BN * SB : BK * SB;
  constexpr int NA = BM * BK / 256, NB = BN * BK / 256;
  // two LDS stages (slice s computes from one while slice s+1 is stored into the other)
  __shared__ __attribute__((aligned(16))) float smem[2 * (LA + LB) + 4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int M = (int)a.M, N = (int)a.N;
  const int Nreal = a.ones_col ? N - 1 : N;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * kchunk;
  int kend = min((int)a.K, kbeg + kchunk);
  if (a.zc_rowptr) {  // empty hop chunks: stop the k loop at their start, or skip whole zero tiles
    const int zE = zc_extent(a.zc_rowptr, a.zc_rows, a.zc_chunks, a.zc_width);
    if (a.zc_dim == 0) {
      kend = min(kend, zE);
    } else if (n0 >= zE && !(a.ones_col && n0 + BN > Nreal)) {  // never the tile of the ones column
      if (blockIdx.z == 0 && a.zc_dim == 1) zero_tile<BM, BN>(a, m0, n0, M, Nreal);  // zc_dim 2: no store
      return;
    }
  }
  const __amdgpu_buffer_rsrc_t ra_ = make_rsrc(a.A, a_bytes);
  const __amdgpu_buffer_rsrc_t rb_ = make_rsrc(a.B, b_bytes);
  const uint32_t sam = (uint32_t)a.sam, sak = (uint32_t)a.sak, sbk = (uint32_t)a.sbk, sbn = (uint32_t)a.sbn;

  // Per-thread fixed coordinates of the staging pattern.
  //  AK : mm = tid / BK + i*(256/BK), kk = tid % BK    |  !AK : mm = tid % BM, kk = tid / BM + i*(256/BM)
  const int a_m = AK ? tid / BK : tid % BM;
  const int a_k = AK ? tid % BK : tid / BM;
  const int b_n = BKC ? tid / BK : tid % BN;
  const int b_k = BKC ? tid % BK : tid / BN;
  constexpr int A_STEP = AK ? 256 / BK : 256 / BM;  // rows (AK) or k (!AK) advanced per i
  constexpr int B_STEP = BKC ? 256 / BK : 256 / BN;
  const bool a_m_ok = AK ? true : (m0 + a_m < M);
  const bool b_n_ok = BKC ? true : (n0 + b_n < Nreal);
  const bool b_n_one = !BKC && a.ones_col && (n0 + b_n == N - 1);

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Epilogue coordinates (the C tile is walked row-major, consecutive lanes on consecutive
  // columns). For tiles with <= 8 outputs per thread, the epilogue operands are loaded NOW so
  // their round trip overlaps the main loop instead of following it (not for split-K launches,
  // where only the last-arriving workgroup runs the epilogue).
  constexpr int NEPI = BM * BN / 256;
  constexpr bool PRE = NEPI <= 8;
  int em[NEPI], en[NEPI];
#pragma unroll
  for (int u = 0; u < NEPI; ++u) {
    const int e = tid + u * 256;
    em[u] = m0 + e / BN;
    en[u] = n0 + e % BN;
  }
  EpiPre<NEPI> epre;
  if constexpr (PRE) {
    if (gridDim.z == 1) epi_load<NEPI>(a, em, en, epre);
  }

  constexpr int NA4 = V4 ? BM * BK / 1024 : 1, NB4 = V4 ? BN * BK / 1024 : 1;
  struct Regs {
    float a[NA];
    float b[NB];
    int k0;  // the slice's first k
  };
  auto load_slice = [&](int k0, bool tail, Regs& R) {
    float(&ra)[NA] = R.a;
    float(&rb)[NB] = R.b;
    R.k0 = k0;
    if constexpr (V4) {
#pragma unroll
      for (int i = 0; i < NA4; ++i) {
        const int q = tid + i * 256;
        const int mm = AK ? q / (BK / 4) : (q % (BM / 4)) * 4;
        const int kk = AK ? (q % (BK / 4)) * 4 : q / (BM / 4);
        const bool ok = (k0 + kk < kend) && (AK || m0 + mm < M);
        const uint32_t off = AK ? 4u * ((uint32_t)(m0 + mm) * sam + (uint32_t)(k0 + kk))
                                : 4u * ((uint32_t)(m0 + mm) + (uint32_t)(k0 + kk) * sak);
        const floatx4 v = bload4(ra_, ok ? off : a_bytes, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[4 * i + e] = v[e];
      }
#pragma unroll
      for (int i = 0; i < NB4; ++i) {
        const int q = tid + i * 256;
        const int nn = BKC ? q / (BK / 4) : (q % (BN / 4)) * 4;
        const int kk = BKC ? (q % (BK / 4)) * 4 : q / (BN / 4);
        const bool kok = k0 + kk < kend;
        const bool ok = kok && (n0 + nn < Nreal);
        const uint32_t off = BKC ? 4u * ((uint32_t)(n0 + nn) * sbn + (uint32_t)(k0 + kk))
                                 : 4u * ((uint32_t)(n0 + nn) + (uint32_t)(k0 + kk) * sbk);
        const floatx4 v = bload4(rb_, ok ? off : b_bytes, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) rb[4 * i + e] = v[e];
      }
      return;
    }
    (void)tail;
    // A
    if (AK) {
      const uint32_t voff = 4u * ((uint32_t)(m0 + a_m) * sam + (uint32_t)(k0 + a_k));
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        ra[i] = bload(ra_, voff, 4u * (uint32_t)(i * A_STEP) * sam);
      }
    } else {
      const uint32_t voff = 4u * ((uint32_t)(m0 + a_m) + (uint32_t)(k0 + a_k) * sak);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        ra[i] = bload(ra_, voff, 4u * (uint32_t)(i * A_STEP) * sak);
      }
    }
    // B
    if (BKC) {
      const uint32_t voff = 4u * ((uint32_t)(n0 + b_n) * sbn + (uint32_t)(k0 + b_k));
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        rb[i] = bload(rb_, voff, 4u * (uint32_t)(i * B_STEP) * sbn);
      }
    } else {
      const uint32_t voff = 4u * ((uint32_t)(n0 + b_n) + (uint32_t)(k0 + b_k) * sbk);
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        rb[i] = bload(rb_, voff, 4u * (uint32_t)(i * B_STEP) * sbk);
      }
    }
  };
  // The validity selects on loaded values (rows / k past the slice's end, the ones column, k past
  // a trimmed kend inside a k-contiguous float4 — zc: 2 D = 306 at c4, where the unwritten next
  // hop chunk begins) are made here, where the data is needed anyway: in load_slice hipcc placed
  // them right after the loads and waited for each load at issue.
  auto store_slice = [&](const Regs& R, int stage) {
    float ra[NA], rb[NB];
    {
      const int k0 = R.k0;
      const bool tail = k0 + BK > kend;
      if constexpr (V4) {
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
          const int q = tid + i * 256;
          const int kk = AK ? (q % (BK / 4)) * 4 : q / (BM / 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) ra[4 * i + e] = (AK && k0 + kk + e >= kend) ? 0.f : R.a[4 * i + e];
        }
#pragma unroll
        for (int i = 0; i < NB4; ++i) {
          const int q = tid + i * 256;
          const int nn = BKC ? q / (BK / 4) : (q % (BN / 4)) * 4;
          const int kk = BKC ? (q % (BK / 4)) * 4 : q / (BN / 4);
          const bool kok = k0 + kk < kend;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool one = a.ones_col && kok && ((BKC ? n0 + nn : n0 + nn + e) == N - 1);
            const bool kin = !BKC || k0 + kk + e < kend;
            rb[4 * i + e] = !kin ? 0.f : (one ? 1.f : R.b[4 * i + e]);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const bool ok = AK ? (!tail || k0 + a_k < kend) : (a_m_ok && (!tail || k0 + a_k + i * A_STEP < kend));
          ra[i] = ok ? R.a[i] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          if (BKC) {
            const bool kok = !tail || k0 + b_k < kend;
            const bool one = a.ones_col && (n0 + b_n + i * B_STEP == N - 1);
            rb[i] = kok ? (one ? 1.f : R.b[i]) : 0.f;
          } else {
            const bool kok = !tail || k0 + b_k + i * B_STEP < kend;
            rb[i] = kok ? (b_n_one ? 1.f : (b_n_ok ? R.b[i] : 0.f)) : 0.f;
          }
        }
      }
    }
    if constexpr (BF) {
      __bf16* Ah = reinterpret_cast<__bf16*>(smem) + stage * (LAH + LBH);
      __bf16* Bh = Ah + LAH;
      if constexpr (V4) {
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
          const int q = tid + i * 256;
          const int mm = AK ? q / (BK / 4) : (q % (BM / 4)) * 4;
          const int kk = AK ? (q % (BK / 4)) * 4 : q / (BM / 4);
          if (AK) {
            *reinterpret_cast<bf16x4*>(&Ah[mm * SH + kk]) =
                bf16x4{(__bf16)ra[4 * i], (__bf16)ra[4 * i + 1], (__bf16)ra[4 * i + 2], (__bf16)ra[4 * i + 3]};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) Ah[(mm + e) * SH + kk] = (__bf16)ra[4 * i + e];
          }
        }
#pragma unroll
        for (int i = 0; i < NB4; ++i) {
          const int q = tid + i * 256;
          const int nn = BKC ? q / (BK / 4) : (q % (BN / 4)) * 4;
          const int kk = BKC ? (q % (BK / 4)) * 4 : q / (BN / 4);
          if (BKC) {
            *reinterpret_cast<bf16x4*>(&Bh[nn * SH + kk]) =
                bf16x4{(__bf16)rb[4 * i], (__bf16)rb[4 * i + 1], (__bf16)rb[4 * i + 2], (__bf16)rb[4 * i + 3]};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) Bh[(nn + e) * SH + kk] = (__bf16)rb[4 * i + e];
          }
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int mm = AK ? a_m + i * A_STEP : a_m;
        const int kk = AK ? a_k : a_k + i * A_STEP;
        Ah[mm * SH + kk] = (__bf16)ra[i];
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int nn = BKC ? b_n + i * B_STEP : b_n;
        const int kk = BKC ? b_k : b_k + i * B_STEP;
        Bh[nn * SH + kk] = (__bf16)rb[i];
      }
      return;
    }
    float* As = smem + stage * (LA + LB);
    float* Bs = As + LA;
    if constexpr (V4) {
#pragma unroll
      for (int i = 0; i < NA4; ++i) {
        const int q = tid + i * 256;
        const int mm = AK ? q / (BK / 4) : (q % (BM / 4)) * 4;
        const int kk = AK ? (q % (BK / 4)) * 4 : q / (BM / 4);
        if (AK) {
#pragma unroll
          for (int e = 0; e < 4; ++e) As[mm * SA + kk + e] = ra[4 * i + e];
        } else {
          *reinterpret_cast<floatx4*>(&As[kk * SA + mm]) =
              floatx4{ra[4 * i], ra[4 * i + 1], ra[4 * i + 2], ra[4 * i + 3]};
        }
      }
#pragma unroll
      for (int i = 0; i < NB4; ++i) {
        const int q = tid + i * 256;
        const int nn = BKC ? q / (BK / 4) : (q % (BN / 4)) * 4;
        const int kk = BKC ? (q % (BK / 4)) * 4 : q / (BN / 4);
        if (BKC) {
#pragma unroll
          for (int e = 0; e < 4; ++e) Bs[nn * SB + kk + e] = rb[4 * i + e];
        } else {
          *reinterpret_cast<floatx4*>(&Bs[kk * SB + nn]) =
              floatx4{rb[4 * i], rb[4 * i + 1], rb[4 * i + 2], rb[4 * i + 3]};
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int mm = AK ? a_m + i * A_STEP : a_m;
      const int kk = AK ? a_k : a_k + i * A_STEP;
      As[AK ? (mm * SA + kk) : (kk * SA + mm)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int nn = BKC ? b_n + i * B_STEP : b_n;
      const int kk = BKC ? b_k : b_k + i * B_STEP;
      Bs[BKC ? (nn * SB + kk) : (kk * SB + nn)] = rb[i];
    }
  };
  auto compute_slice = [&](int stage) {
    if constexpr (BF) {
      const __bf16* Ah = reinterpret_cast<const __bf16*>(smem) + stage * (LAH + LBH);
      const __bf16* Bh = Ah + LAH;
      bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(&Ah[(wr * WM + i * 16 + (lane & 15)) * SH + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[j] = *reinterpret_cast<const bf16x8*>(&Bh[(wc * WN + j * 16 + (lane & 15)) * SH + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      return;
    }
    const float* As = smem + stage * (LA + LB);
    const float* Bs = As + LA;
    auto rd = [&](int s, float (&af)[TM], float (&bf)[TN]) {
      const int kr = 4 * s + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mm = wr * WM + i * 16 + (lane & 15);
        af[i] = As[AK ? (mm * SA + kr) : (kr * SA + mm)];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nn = wc * WN + j * 16 + (lane & 15);
        bf[j] = Bs[BKC ? (nn * SB + kr) : (kr * SB + nn)];
      }
    };
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      float af[TM], bf[TN];
      rd(s, af, bf);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  // Software pipeline: two register sets and two LDS stages. While slice s is multiplied from
  // LDS, slice s+1 waits in registers (its loads were issued one slice earlier) and slice s+2's
  // loads are in flight, so each global load has two slices of MFMA work to land behind.
  const int nsl = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  Regs r0, r1;
  if (nsl > 0) load_slice(kbeg, kbeg + BK > kend, r0);
  if (nsl > 1) load_slice(kbeg + BK, kbeg + 2 * BK > kend, r1);
  if (nsl > 0) store_slice(r0, 0);
  __syncthreads();
  // The loads run unconditionally (a slice past the end is never stored): under a condition, the
  // two paths into the next wait carry different pending loads and hipcc waits for all of them
  // (vmcnt(0)) before each store_slice, including the slice issued just before the compute.
  for (int sl = 0; sl < nsl; sl += 2) {
    {
      const int k2 = kbeg + (sl + 2) * BK;
      load_slice(k2, k2 + BK > kend, r0);
    }
    compute_slice(0);
    if (sl + 1 < nsl) store_slice(r1, 1);
    __syncthreads();
    if (sl + 1 >= nsl) break;
    {
      const int k3 = kbeg + (sl + 3) * BK;
      load_slice(k3, k3 + BK > kend, r1);
    }
    compute_slice(1);
    if (sl + 2 < nsl) store_slice(r0, 0);
    __syncthreads();
  }

  if (gridDim.z > 1) {
    // ---- split-K: this slice's partial tile goes to a slab in ACCUMULATOR order (thread tid's
    // float4 for fragment (i, j) at ((i*TN + j)*256 + tid)*4), so slab writes and the reducer's
    // reads are contiguous 16-B-per-lane streams ----
    const int tile = blockIdx.x * gridDim.y + blockIdx.y;
    const int64_t ntiles = (int64_t)gridDim.x * gridDim.y;
    constexpr int TILE = BM * BN;
    const int S = (int)gridDim.z;
    const __amdgpu_buffer_rsrc_t rws = make_rsrc(a.workspace, (uint32_t)(4 * (int64_t)S * ntiles * TILE));
    const uint32_t slab0 = (uint32_t)(4 * (((int64_t)blockIdx.z * ntiles + tile) * TILE));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) store_sc1(rws, slab0 + 16u * (uint32_t)((i * TN + j) * 256 + tid), acc[i][j]);
    if (!a.counters) return;  // reduced by k_splitk_reduce
    // ---- in-launch ordered reduce by the last arriver (sc1 hand-off, see store_sc1) ----
    int* flag = reinterpret_cast<int*>(smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(&a.counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (old == S - 1);
      if (last) __hip_atomic_store(&a.counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // self-reset
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    // slabs summed in slice order (deterministic), 8 slices' float4 loads in flight per fragment
    const uint32_t zstride = (uint32_t)(4 * ntiles * TILE);  // bytes per slice
    const uint32_t tile0 = (uint32_t)(4 * (int64_t)tile * TILE);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const uint32_t off = tile0 + 16u * (uint32_t)((i * TN + j) * 256 + tid);
        floatx4 s = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int z0 = 0; z0 < S; z0 += 8) {
          floatx4 t[8];
#pragma unroll
          for (int w = 0; w < 8; ++w) t[w] = load_sc1(rws, (uint32_t)min(z0 + w, S - 1) * zstride + off);
#pragma unroll
          for (int w = 0; w < 8; ++w)
            if (z0 + w < S) s += t[w];
        }
        acc[i][j] = s;
      }
  }

  // C/D layout of the 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg. The tile is
  // transposed through LDS so the epilogue walks rows with consecutive lanes on consecutive
  // columns: coalesced residual/bias/mask loads and C/pre stores (4 elements per thread per pass).
  {
    constexpr int CS = BN + 1;
    static_assert(BM * CS <= 2 * (LA + LB), "C tile must fit the staging LDS");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          smem[(wr * WM + i * 16 + (lane >> 4) * 4 + r) * CS + wc * WN + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();
    if constexpr (PRE) {
      float ev[NEPI];
#pragma unroll
      for (int u = 0; u < NEPI; ++u) {
        const int e = tid + u * 256;
        ev[u] = smem[(e / BN) * CS + e % BN];
      }
      if (gridDim.z > 1) epi_load<NEPI>(a, em, en, epre);
      epi_apply<NEPI>(a, em, en, ev, epre);
    } else {
      // chunks of 8 outputs, each chunk's epilogue operands in flight together (one round trip
      // per chunk: 2 for a 64x64 tile, was 4 with chunks of 4; all 16 at once needs ~200 VGPRs)
#pragma unroll
      for (int q0 = 0; q0 < NEPI; q0 += 8) {
        int qm[8], qn[8];
        float ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int e = tid + (q0 + u) * 256;
          qm[u] = em[q0 + u];
          qn[u] = en[q0 + u];
          ev[u] = smem[(e / BN) * CS + e % BN];
        }
        epilogue_n<8>(a, qm, qn, ev);
      }
    }
  }
}

// 32 x 32 x 2 fp32 MFMA accumulator (k_gemm_deep)
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---- Weight-gradient GEMM (K = atoms, small M x N): MFMA fragments straight from L2 ----------
// dW = dY^T X: A = dY^T is m-contiguous (sam == 1), B = X is n-contiguous (sbn == 1), K is the atom
// count. In that layout the 16x16x4 MFMA fragments ARE coalesced global rows (lane l reads A[k0 +
// l/16][m0 + l%16], 16 consecutive floats per k), so each wave loads its own fragments with no
// LDS staging and no barriers, keeping kWgU k-steps (8 x 4 fragment loads per lane) in flight.
// A workgroup owns one 32x32 output tile; its 4 waves split the workgroup's K range in 4 and are
// summed through LDS in wave order; workgroups split K further (split-K slabs + ordered
// last-arriver reduce, as in k_gemm). Deterministic throughout.
constexpr int kWgU = 8;

// One 32x32 output tile, K slice bz of S (of width kchunk): the body shared by the single-problem
// kernel and the grouped one. Slabs of this problem live at ws + (z * ntiles + tile) * 1024.
__device__ __forceinline__ void wgrad_block(const AimxGemmArgs& a, int kchunk, uint32_t a_bytes, uint32_t b_bytes,
                                            int bx, int by, int bz, int S, int tile, int ntiles, float* ws,
                                            int32_t* counters, float* red) {
  // the wave index is made provably uniform so the k-dependent buffer offsets stay scalar (SGPR
  // soffset); otherwise hipcc waterfalls every fragment load
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = (int)a.M, N = (int)a.N;
  const int m0 = bx * 32, n0 = by * 32;
  if (a.zc_rowptr) {  // a tile wholly inside the empty hop chunks: zero gradient, no work
    const int Nreal = a.ones_col ? N - 1 : N;
    if (n0 >= zc_extent(a.zc_rowptr, a.zc_rows, a.zc_chunks, a.zc_width) && !(a.ones_col && n0 + 32 > Nreal)) {
      if (bz == 0) zero_tile<32, 32>(a, m0, n0, M, Nreal);
      return;
    }
  }
  const int kb = bz * kchunk;
  const int kend = min((int)a.K, kb + kchunk);
  const int kw = kchunk / 4;  // multiple of 4
  const int k0 = min(kend, kb + w * kw), k1 = min(kend, kb + (w + 1) * kw);
  const __amdgpu_buffer_rsrc_t ra_ = make_rsrc(a.A, a_bytes);
  const __amdgpu_buffer_rsrc_t rb_ = make_rsrc(a.B, b_bytes);
  const uint32_t sak = (uint32_t)a.sak, sbk = (uint32_t)a.sbk;
  const int lm = lane & 15, lk = lane >> 4;
  // X columns in the trailing empty hop chunks (zc) read as zero: the stack's hop does not write
  // them (segment_gather_sum skip_tail), and their exact gradient is zero
  const int zlim = a.zc_rowptr ? zc_extent(a.zc_rowptr, a.zc_rows, a.zc_chunks, a.zc_width) : N;
  uint32_t va[2], vb[2];
  bool one[2], zcol[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    va[i] = 4u * ((uint32_t)(m0 + i * 16 + lm) + (uint32_t)lk * sak);
    vb[i] = 4u * ((uint32_t)(n0 + i * 16 + lm) + (uint32_t)lk * sbk);
    one[i] = a.ones_col && (n0 + i * 16 + lm == N - 1);
    zcol[i] = !one[i] && n0 + i * 16 + lm >= zlim;
  }
  floatx4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // k beyond the wave's range: the per-lane offset is moved past the descriptor's extent, so the
  // (unconditional) load returns 0 — a select on the address, never on the loaded value, keeps
  // every load of the group in flight (a value select lets hipcc sink loads under a branch)
  auto load_group = [&](int kg, float (&fa)[kWgU][2], float (&fb)[kWgU][2]) {
#pragma unroll
    for (int u = 0; u < kWgU; ++u) {
      const int kk = kg + 4 * u;
      const bool kok = kk + lk < k1;
      const uint32_t sa = __builtin_amdgcn_readfirstlane(4u * (uint32_t)kk * sak);
      const uint32_t sb = __builtin_amdgcn_readfirstlane(4u * (uint32_t)kk * sbk);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[u][i] = bload(ra_, kok ? va[i] : a_bytes, sa);
        // raw: the ones column is substituted where the value is consumed (mma_group) — a select
        // here made hipcc wait for this group's loads before the previous group's MFMAs
        fb[u][i] = bload(rb_, kok && !zcol[i] ? vb[i] : b_bytes, sb);
      }
    }
  };
  auto mma_group = [&](const float (&fa)[kWgU][2], const float (&fb)[kWgU][2]) {
#pragma unroll
    for (int u = 0; u < kWgU; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float b = one[j] ? 1.f : fb[u][j];  // (fa is 0 on rows past the wave's k range)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[u][i], b, acc[i][j], 0, 0, 0);
        }
  };
  constexpr int KG = 4 * kWgU;
  const int ng = k1 > k0 ? (k1 - k0 + KG - 1) / KG : 0;
  float fa0[kWgU][2], fb0[kWgU][2], fa1[kWgU][2], fb1[kWgU][2];
  if (ng > 0) load_group(k0, fa0, fb0);
  // loads unconditional (a group past the range reads 0): conditional ones leave hipcc waiting
  // for every load at the loop head
  for (int g = 0; g < ng; g += 2) {
    load_group(k0 + (g + 1) * KG, fa1, fb1);
    mma_group(fa0, fb0);
    if (g + 1 >= ng) break;
    load_group(k0 + (g + 2) * KG, fa0, fb0);
    mma_group(fa1, fb1);
  }
  // intra-workgroup K reduction, wave order 0,1,2,3 (deterministic)
  if (w > 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<floatx4*>(&red[(w - 1) * 1024 + ((i * 2 + j) * 64 + lane) * 4]) = acc[i][j];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] += *reinterpret_cast<const floatx4*>(&red[q * 1024 + ((i * 2 + j) * 64 + lane) * 4]);
  }
  if (S > 1) {
    const __amdgpu_buffer_rsrc_t rws = make_rsrc(ws, (uint32_t)(4 * (int64_t)S * ntiles * 1024));
    const uint32_t slab0 = (uint32_t)(4 * (((int64_t)bz * ntiles + tile) * 1024));
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) store_sc1(rws, slab0 + 16u * (uint32_t)((i * 2 + j) * 64 + lane), acc[i][j]);
    }
    if (!counters) return;
    // sc1 hand-off (see store_sc1): drained stores -> barrier -> one agent add; last adder reduces
    int* flag = reinterpret_cast<int*>(red);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(&counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (old == S - 1);
      if (last) __hip_atomic_store(&counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // self-reset
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    // ordered slab sum: wave q sums slices q, q+4, ... ; the 4 partial sums are added in wave order
    const uint32_t zs = (uint32_t)(4 * ntiles * 1024);  // bytes per slice
    const uint32_t tile0 = (uint32_t)(4 * (int64_t)tile * 1024);
    floatx4 part[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t off = tile0 + 16u * (uint32_t)((i * 2 + j) * 64 + lane);
        floatx4 sum = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int z0 = w; z0 < S; z0 += 16) {
          floatx4 t[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) t[q] = load_sc1(rws, (uint32_t)min(z0 + 4 * q, S - 1) * zs + off);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (z0 + 4 * q < S) sum += t[q];
        }
        part[i][j] = sum;
      }
    __syncthreads();
    if (w > 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<floatx4*>(&red[(w - 1) * 1024 + ((i * 2 + j) * 64 + lane) * 4]) = part[i][j];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = part[i][j];
#pragma unroll
          for (int q = 0; q < 3; ++q)
            acc[i][j] += *reinterpret_cast<const floatx4*>(&red[q * 1024 + ((i * 2 + j) * 64 + lane) * 4]);
        }
    }
  }
  // epilogue: wave 0's tile -> LDS (row-major, stride 33) -> all 256 threads, 4 elements each
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(i * 16 + lk * 4 + r) * 33 + j * 16 + lm] = acc[i][j][r];
  }
  __syncthreads();
  int em[4], en[4];
  float ev[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + u * 256;
    em[u] = m0 + e / 32;
    en[u] = n0 + e % 32;
    ev[u] = red[(e / 32) * 33 + e % 32];
  }
  (void)M;
  epilogue_n<4>(a, em, en, ev);
}

__global__ __launch_bounds__(256) void k_wgrad(const AimxGemmArgs a, int kchunk, uint32_t a_bytes, uint32_t b_bytes) {
  __shared__ __attribute__((aligned(16))) float red[3 * 1024];
  wgrad_block(a, kchunk, a_bytes, b_bytes, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.z,
              blockIdx.x * gridDim.y + blockIdx.y, gridDim.x * gridDim.y, a.workspace, a.counters, red);
}

// Grouped weight gradients: up to kWgMaxProb independent dW = dY^T X problems in one launch (the
// whole message-passing stack's weight gradients, deferred to the end of its backward), so the
// per-launch latency of ~15 small long-K GEMMs is paid once and their workgroups fill the chip.
constexpr int kWgMaxProb = 16;
struct WgradTable {
  int32_t n;
  int32_t blk0[kWgMaxProb + 1];  // first workgroup of each problem
  int32_t tiles_y[kWgMaxProb], ntiles[kWgMaxProb], splits[kWgMaxProb], kchunk[kWgMaxProb];
  uint32_t a_bytes[kWgMaxProb], b_bytes[kWgMaxProb];
  int64_t ws_off[kWgMaxProb], cnt_off[kWgMaxProb];
  AimxWgradProblem p[kWgMaxProb];
};

__global__ __launch_bounds__(256) void k_wgrad_grouped(const WgradTable t, float* ws, int32_t* counters) {
  __shared__ __attribute__((aligned(16))) float red[3 * 1024];
  int q = 0;
  while (q + 1 < t.n && t.blk0[q + 1] <= (int)blockIdx.x) ++q;
  const int local = blockIdx.x - t.blk0[q];
  const int nt = t.ntiles[q];
  const int z = local / nt, tile = local - z * nt;
  const AimxWgradProblem& pr = t.p[q];
  AimxGemmArgs a = {};
  a.M = pr.M;
  a.N = pr.col_out ? pr.N + 1 : pr.N;
  a.K = pr.K;
  a.A = pr.dY;
  a.sam = 1;
  a.sak = pr.ld_dy;
  a.B = pr.X;
  a.sbk = pr.ld_x;
  a.sbn = 1;
  a.C = pr.dW;
  a.ldc = pr.ld_dw;
  a.act = -1;
  a.dact_kind = -1;
  a.ones_col = pr.col_out ? 1 : 0;
  a.col_out = pr.col_out;
  a.zc_rowptr = pr.zc_rowptr;
  a.zc_rows = pr.zc_rows;
  a.zc_chunks = pr.zc_chunks;
  a.zc_width = pr.zc_width;
  a.zc_dim = 1;
  wgrad_block(a, t.kchunk[q], t.a_bytes[q], t.b_bytes[q], tile / t.tiles_y[q], tile % t.tiles_y[q], z, t.splits[q],
              tile, nt, ws + t.ws_off[q], counters ? counters + t.cnt_off[q] : nullptr, red);
}

// ---- Long-K weight gradients through LDS: 64 x 64 or 80 x 80 output blocks ---------------------
// k_wgrad_grouped's waves load their MFMA fragments straight from global memory: one dword load
// per MFMA, re-read by every 32 x 32 tile of the output, which leaves that kernel address-rate
// bound (~30 % MFMA issue). Here a workgroup owns a BB x BB block (80: a whole 76 x 76 + bias MLP
// weight of c2, or a quarter of its input projection; 64: four waves, one per SIMD) and a K slice:
// 32 k rows of dY and X are staged in LDS by 16-byte loads (each element read once per block) in two
// LDS buffers, prefetched into registers while the previous rows compute; wave w (of BB / 16) owns
// fragment row w and runs its BB / 16 MFMAs per k step from LDS (A read once, reused across the
// row). LDS row strides of 80 floats put the 4 k rows of a fragment read on bank offsets 0/16/32/48:
// conflict-free. Split-K slices are summed as in k_wgrad_grouped (sc1 slabs, last arriver adds
// them in slice order): deterministic.
constexpr int kWbK = 32;                             // k rows per LDS fill
constexpr int kWbD = 2;                              // LDS fills in flight (register ring)
template <int BB>
struct WbGeom {
  static constexpr int F = BB / 16;                  // fragments per edge = waves per workgroup
  static constexpr int T = 64 * F;                   // threads per workgroup
  static constexpr int S = BB == 80 ? 80 : BB + 16;  // LDS row stride (floats)
  static constexpr int Slab = BB * BB;               // floats per split-K slab
  static constexpr int Q = kWbK * BB / 4;            // float4 per operand per fill
  static constexpr int V = 2 * Q / T;                // float4 per thread per fill
  static_assert(Q % T == 0, "each thread's float4s belong to one operand");
};

struct WbTable {
  int32_t n;
  int32_t blk0[kWgMaxProb + 1];
  int32_t bn[kWgMaxProb], nblk[kWgMaxProb], splits[kWgMaxProb], kchunk[kWgMaxProb], v4[kWgMaxProb];
  uint32_t a_bytes[kWgMaxProb], b_bytes[kWgMaxProb];
  int64_t ws_off[kWgMaxProb], cnt_off[kWgMaxProb];
  AimxWgradProblem p[kWgMaxProb];
  int32_t xcd;  // XCD-aware work order
};

#ifdef AIMX_WB_TRACE  // diagnostics build only: per-wave shader-clock totals of k_wgrad_lds phases
// [traced workgroup][wave][phase: put (waits for the fill's loads), fetch (issue), compute, barrier, total]
__device__ long long g_wb_trace[4][10][5];
#define WBT(slot, stmt)                                         \
  do {                                                          \
    const long long t0_ = (long long)__builtin_readcyclecounter(); \
    stmt;                                                       \
    wbt[slot] += (long long)__builtin_readcyclecounter() - t0_; \
  } while (0)
#else
#define WBT(slot, stmt) stmt
#endif

// Two LDS buffers per operand (40 KiB at 80 wide: four workgroups fill a CU's 160 KiB). Fill s + 1 is written to the idle buffer while fill s computes from the other, so each
// fill costs one workgroup barrier instead of two and the LDS writes overlap other waves' MFMAs.
// VM: the operands' staging, 1 = 16-byte loads for every problem of the launch, 0 = dword loads for
// every problem, 2 = per problem (WbTable.v4). With a per-problem branch inside each fetch the
// paths into the fill loop's head carry different load counts and hipcc waits for all loads there.
// 80-wide blocks: 5 waves per SIMD (<= 102 VGPRs), so that four workgroups (20 waves, all the LDS)
// fit a CU; at 108-112 VGPRs only three did
template <int BB, int VM>
__global__ __launch_bounds__(WbGeom<BB>::T) __attribute__((amdgpu_waves_per_eu(BB == 80 ? 5 : 1)))
void k_wgrad_lds(const WbTable t, float* ws, int32_t* counters) {
  using G = WbGeom<BB>;
  constexpr int kWbF = G::F, kWbT = G::T, kWbV = G::V, kLd = G::S;
  constexpr int kBuf = kWbK * kLd;  // floats per operand buffer
  __shared__ __attribute__((aligned(16))) float sA[2 * kBuf];
  __shared__ __attribute__((aligned(16))) float sB[2 * kBuf];
  // the split-K arrival flag lives in sA: written only after the barrier that ends every LDS read
  int& flag = *reinterpret_cast<int*>(sA);
  int q = 0;
  while (q + 1 < t.n && t.blk0[q + 1] <= (int)blockIdx.x) ++q;
  const int nb = t.nblk[q];
  int local = blockIdx.x - t.blk0[q];
  // XCD-aware work order: blocks b and b + 8 share an XCD (and its L2). The problem's work items
  // (split-major, output blocks fastest) are dealt in 8 contiguous runs, one per XCD, so the nb
  // blocks that read the same K slice of dY and X run on one XCD and share its L2 instead of
  // fetching the slice once per XCD. Only the first floor(items/8)*8 items move. Speed only.
  // Measured (profiles/r02_wgrad_xcd_ab.txt): c2 -12 us, c4 -30 us per step; with c5's 64 blocks
  // per K slice it was 35 us slower, so problems with more than 32 blocks keep the launch order.
  if (t.xcd && nb <= 32) {
    const int items = nb * t.splits[q], i8 = items & ~7;
    if (local < i8) local = (local & 7) * (i8 >> 3) + (local >> 3);
  }
  const int z = local / nb, blk = local - z * nb;
  const AimxWgradProblem& pr = t.p[q];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lm = lane & 15, lk = lane >> 4;
  const int M = (int)pr.M, Nreal = (int)pr.N, ones = pr.col_out != nullptr;
  const int N = Nreal + ones;
  const int m0 = (blk / t.bn[q]) * BB, n0 = (blk % t.bn[q]) * BB;
  const int S = t.splits[q];
  AimxGemmArgs a = {};
  a.M = M;
  a.N = N;
  a.K = pr.K;
  a.C = pr.dW;
  a.ldc = pr.ld_dw;
  a.act = -1;
  a.dact_kind = -1;
  a.ones_col = ones;
  a.col_out = pr.col_out;
  // X columns in the trailing empty hop chunks read as zero (see wgrad_block)
  const int zlim = pr.zc_rowptr ? min(Nreal, zc_extent(pr.zc_rowptr, pr.zc_rows, pr.zc_chunks, pr.zc_width)) : Nreal;
  if (pr.zc_rowptr && n0 >= zlim && !(ones && n0 + BB > Nreal)) {  // a block wholly inside the empty hop chunks: zero, no work
    if (z == 0)
      for (int e = tid; e < G::Slab; e += kWbT) {
        const int m = m0 + e / BB, n = n0 + e % BB;
        if (m < M && n < Nreal) pr.dW[(int64_t)m * pr.ld_dw + n] = 0.f;
      }
    return;
  }
  const int kb = z * t.kchunk[q];
  const int kend = min((int)pr.K, kb + t.kchunk[q]);
  const int nsub = kend > kb ? (kend - kb + kWbK - 1) / kWbK : 0;
  // descriptors over this split's K rows only (32-bit offsets from the split's first row: a problem
  // of any K stays addressable; wg_plan keeps one split's rows under 2 GiB)
  const uint32_t ab = t.a_bytes[q], bb = t.b_bytes[q];
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(pr.dY + (int64_t)kb * pr.ld_dy, ab);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(pr.X + (int64_t)kb * pr.ld_x, bb);
  const uint32_t lda = (uint32_t)pr.ld_dy, ldb = (uint32_t)pr.ld_x;
  const bool v4 = VM == 2 ? t.v4[q] != 0 : VM == 1;

  // rows k0.. of both operands -> registers: loads only, every validity test an ADDRESS select
  // (rows past kend and float4s wholly past the column limit point past the descriptor's extent
  // and read 0). A value select here — zeroing the components of a float4 that straddles the limit,
  // or writing X's implicit ones column — made hipcc wait for each load right after issuing it
  // (a branch per load: cdna_hip_programming.md §5 trap (c)), so no fill was ever in flight during
  // the compute; those selects run in put, where the data is needed anyway.
  auto fetch = [&](int k0, floatx4 (&stage)[kWbV]) {
#pragma unroll
    for (int u = 0; u < kWbV; ++u) {
      const bool isb = u >= kWbV / 2;
      const int f = tid + (isb ? u - kWbV / 2 : u) * kWbT;
      const int row = f / (BB / 4), c = 4 * (f % (BB / 4));
      const int k = k0 + row, kr = k - kb;  // kr: row within the split (the descriptors' base)
      const int col = (isb ? n0 : m0) + c, lim = isb ? zlim : M;
      const uint32_t ld = isb ? ldb : lda, bytes = isb ? bb : ab;
      const __amdgpu_buffer_rsrc_t r = isb ? rb : ra;
      const bool kok = k < kend;
      floatx4 v;
      if (v4) {
        v = bload4(r, kok && col < lim ? 4u * ((uint32_t)kr * ld + (uint32_t)col) : bytes, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          v[i] = bload(r, kok && col + i < lim ? 4u * ((uint32_t)kr * ld + (uint32_t)(col + i)) : bytes, 0);
      }
      stage[u] = v;
    }
  };

  floatx4 acc[kWbF];
#pragma unroll
  for (int j = 0; j < kWbF; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 ring[kWbD][kWbV];
  // fill (rows k0..) in registers -> LDS buffer (sa, sb): components of a float4 straddling the
  // column limit are zeroed, X's implicit ones column (the bias gradient) reads 1 on valid rows
  auto put = [&](const floatx4(&stage)[kWbV], int k0, float* sa, float* sb) {
#pragma unroll
    for (int u = 0; u < kWbV; ++u) {
      const bool isb = u >= kWbV / 2;
      const int f = tid + (isb ? u - kWbV / 2 : u) * kWbT;
      const int row = f / (BB / 4), c = 4 * (f % (BB / 4));
      const int col = (isb ? n0 : m0) + c, lim = isb ? zlim : M;
      const bool kok = k0 + row < kend;
      floatx4 v = stage[u];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (v4 && col + i >= lim) v[i] = 0.f;
        if (isb && ones && kok && col + i == Nreal) v[i] = 1.f;
      }
      *reinterpret_cast<floatx4*>((isb ? sb : sa) + row * kLd + c) = v;
    }
  };
  // the kWbK k rows staged in (sa, sb) into this wave's accumulators
  auto compute = [&](const float* sa, const float* sb) {
#pragma unroll
    for (int k4 = 0; k4 < kWbK / 4; ++k4) {
      const int r = (k4 * 4 + lk) * kLd + lm;
      const float av = sa[r + w * 16];
      float bv[kWbF];
#pragma unroll
      for (int j = 0; j < kWbF; ++j) bv[j] = sb[r + j * 16];
#pragma unroll
      for (int j = 0; j < kWbF; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[j], acc[j], 0, 0, 0);
    }
  };
#ifdef AIMX_WB_TRACE
  long long wbt[5] = {0, 0, 0, 0, 0};
  const long long wbt0 = (long long)__builtin_readcyclecounter();
#endif
#pragma unroll
  for (int d = 0; d < kWbD; ++d)
    fetch(kb + d * kWbK, ring[d]);
  static_assert(kWbD == 2, "the double-buffered schedule keeps two fills in registers");
  // fill s computes from buffer s & 1; fill s + 1 (loaded two compute periods earlier) goes to
  // the other buffer first, and its register slot is refilled with fill s + 3
  WBT(0, put(ring[0], kb, sA, sB));
  WBT(1, fetch(kb + 2 * kWbK, ring[0]));
  WBT(3, __syncthreads());
  // put and fetch run unconditionally (fills past the slice are zeros, put into the idle
  // buffer): with them under a condition, the paths into the loop head differ in their pending
  // loads and hipcc waits for all of them there (vmcnt(0)), ending every fill's prefetch
  // (sched_barrier: the fills' loads issue before the compute; hipcc would sink them below it)
  for (int s0 = 0; s0 < nsub; s0 += 2) {
    WBT(0, put(ring[1], kb + (s0 + 1) * kWbK, sA + kBuf, sB + kBuf));
    WBT(1, fetch(kb + (s0 + 3) * kWbK, ring[1]));
    __builtin_amdgcn_sched_barrier(0);
    WBT(2, compute(sA, sB));
    WBT(3, __syncthreads());  // fill s0 + 1 visible; every read of buffer 0 done before it is refilled
    if (s0 + 1 >= nsub) break;
    WBT(0, put(ring[0], kb + (s0 + 2) * kWbK, sA, sB));
    WBT(1, fetch(kb + (s0 + 4) * kWbK, ring[0]));
    __builtin_amdgcn_sched_barrier(0);
    WBT(2, compute(sA + kBuf, sB + kBuf));
    WBT(3, __syncthreads());
  }

#ifdef AIMX_WB_TRACE
  {
    const int slot = blockIdx.x == 0 ? 0 : blockIdx.x == 777 ? 1 : blockIdx.x == 2222 ? 2 : blockIdx.x == 4444 ? 3 : -1;
    wbt[4] = (long long)__builtin_readcyclecounter() - wbt0;
    if (slot >= 0 && lane == 0 && w < 10)
      for (int i = 0; i < 5; ++i) __builtin_nontemporal_store(wbt[i], &g_wb_trace[slot][w][i]);
  }
#endif
  if (S > 1) {
    const __amdgpu_buffer_rsrc_t rws = make_rsrc(ws + t.ws_off[q], (uint32_t)(4 * (int64_t)S * nb * G::Slab));
    const uint32_t own = 16u * (uint32_t)((w * kWbF) * 64 + lane);
#pragma unroll
    for (int j = 0; j < kWbF; ++j)
      store_sc1(rws, 4u * (uint32_t)((z * nb + blk) * G::Slab) + own + 16u * 64u * (uint32_t)j, acc[j]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int32_t* cnt = counters + t.cnt_off[q] + blk;
      const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (old == S - 1);
      if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // self-reset
      flag = last;
    }
    __syncthreads();
    if (!flag) return;
#pragma unroll
    for (int j = 0; j < kWbF; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int zz = 0; zz < S; ++zz) {  // slice order
      floatx4 v[kWbF];
#pragma unroll
      for (int j = 0; j < kWbF; ++j)
        v[j] = load_sc1(rws, 4u * (uint32_t)((zz * nb + blk) * G::Slab) + own + 16u * 64u * (uint32_t)j);
#pragma unroll
      for (int j = 0; j < kWbF; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < kWbF; ++j) {
    int em[4], en[4];
    float ev[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      em[r] = m0 + w * 16 + lk * 4 + r;
      en[r] = n0 + j * 16 + lm;
      ev[r] = acc[j][r];
    }
    epilogue_n<4>(a, em, en, ev);
  }
}

// Fallback when no counter array is supplied: one thread per output element sums the slabs in
// slice order. Slab element (m, n) of tile (tm, tn) sits where thread tid's accumulator fragment
// put it (see the split-K branch of k_gemm).
template <int BM, int BN>
__global__ void k_splitk_reduce(const AimxGemmArgs a, int splits, int tiles_n) {
  constexpr int WM = BM / 2, WN = BN / 2, TN = WN / 16;
  const int64_t total = a.M * a.N;
  const int64_t ntiles = (int64_t)((a.M + BM - 1) / BM) * tiles_n;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(t / a.N), n = (int)(t % a.N);
    const int tile = (m / BM) * tiles_n + n / BN;
    const int lm = m % BM, ln = n % BN;
    const int wr = lm / WM, wc = ln / WN, i = (lm % WM) / 16, j = (ln % WN) / 16;
    const int r = lm % 4, lane = ((lm % 16) / 4) * 16 + (ln % 16);
    const int tid = (wr * 2 + wc) * 64 + lane;
    const int64_t off = ((int64_t)((i * TN + j) * 256 + tid)) * 4 + r;
    float v[1] = {0.f};
    for (int z = 0; z < splits; ++z) v[0] += a.workspace[((int64_t)z * ntiles + tile) * (BM * BN) + off];
    const int mm[1] = {m}, nn[1] = {n};
    epilogue_n<1>(a, mm, nn, v);
  }
}

// ---- Few rows, deep K: the post-pool chain's G x F x F products (k_gemm_deep) ------------------
// c5's head runs G = 256 molecules through F = 1024 square Linears (gnn.py:252-258): 256 32 x 32
// output tiles, one per CU, K = 1024. Staged through LDS (k_gemm<32,32>, split K) every k slice
// waits a full L2 round trip behind a barrier: ~14 us per GEMM at ~15 % MFMA. Here a workgroup of
// 8 waves owns one 32 x 32 tile and every wave computes the WHOLE tile over 1/8 of K with
// v_mfma_f32_32x32x2_f32, loading its fragments straight from L2 into a register ring (no LDS
// staging, no barrier until the end): A (k-contiguous) and B as [n][k] come as one 16-byte load per
// lane per 8 k (lane half h holds k = 8g + 4h + j for MFMA j: the same permutation on both
// operands, so the products pair up), B as [k][n] (the input gradient's W) as one coalesced dword
// per lane per MFMA. The 8 partial tiles meet in LDS and are summed in wave order (deterministic);
// the epilogue operands are loaded before the k loop.
constexpr int kDpU = 4;  // 8-k groups per register set (two sets alternate: 8 groups in flight)

template <bool BKC, int NW>
__global__ __launch_bounds__(64 * NW) void k_gemm_deep(const AimxGemmArgs a, int tiles_m, int ntiles, int kq,
                                                       uint32_t a_bytes, uint32_t b_bytes) {
  constexpr int NO = 1024 / (64 * NW);  // outputs finished per thread
  __shared__ __attribute__((aligned(16))) float red[NW * 1024];
  // XCD-aware order: the blocks of one XCD (b % 8 under round-robin dispatch) take a contiguous
  // range of tiles, column-tile major, so an XCD's L2 holds 1/8 of B (bijective for any grid)
  const int bid = blockIdx.x, nb = (int)gridDim.x;
  const int q = nb / 8, rr = nb % 8, xcd = bid % 8, loc = bid / 8;
  const int tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  if (tile >= ntiles) return;
  const int m0 = (tile % tiles_m) * 32, n0 = (tile / tiles_m) * 32;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int M = (int)a.M, N = (int)a.N, K = (int)a.K;

  // this thread's NO outputs (tile element NO t + u: row / 32, column % 32); their epilogue operands
  // are loaded now, raw and branch-free (an absent operand is a 0-byte descriptor: its loads return
  // 0), and combined after the k loop exactly as epi_load does: nothing waits for them before then
  const int er = (NO * tid) >> 5, ec = (NO * tid) & 31;
  int em[NO], en[NO];
#pragma unroll
  for (int u = 0; u < NO; ++u) em[u] = m0 + er, en[u] = n0 + ec + u;
  float ec_c[NO], ec_b[NO], ec_r[3][NO], ec_p[NO];
  uint32_t ec_k[NO];
  {
    auto ext = [&](const void* p, int64_t ld) { return p ? (uint32_t)(4 * ((a.M - 1) * ld + a.N)) : 0u; };
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(a.C, a.beta != 0.f ? ext(a.C, a.ldc) : 0u);
    const __amdgpu_buffer_rsrc_t rbias = make_rsrc(a.bias, a.bias ? (uint32_t)(4 * a.N) : 0u);
    const __amdgpu_buffer_rsrc_t rp = make_rsrc(a.dact_pre, ext(a.dact_pre, a.lddact));
    const __amdgpu_buffer_rsrc_t rk =
        make_rsrc(a.mask_in, a.mask_in ? (uint32_t)((a.M - 1) * a.ldmask + a.N) : 0u);
#pragma unroll
    for (int e = 0; e < NO; ++e) {
      const bool in = (em[e] < M) & (en[e] < N);
      const uint32_t me = (uint32_t)em[e], ne = (uint32_t)en[e];
      ec_c[e] = bload(rc, in ? 4u * (me * (uint32_t)a.ldc + ne) : kBufDrop, 0);
      ec_b[e] = bload(rbias, in ? 4u * ne : kBufDrop, 0);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.res[q], ext(a.res[q], a.ldres[q]));
        ec_r[q][e] = bload(rr, in ? 4u * (me * (uint32_t)a.ldres[q] + ne) : kBufDrop, 0);
      }
      ec_p[e] = bload(rp, in ? 4u * (me * (uint32_t)a.lddact + ne) : kBufDrop, 0);
      ec_k[e] = __builtin_amdgcn_raw_buffer_load_b8(rk, in ? me * (uint32_t)a.ldmask + ne : kBufDrop, 0, 0);
    }
  }

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.A, a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(a.B, b_bytes);
  const int kb = min(K, w * kq), ke = min(K, kb + kq);
  const uint32_t lda = (uint32_t)a.sam, ldb = BKC ? (uint32_t)a.sbn : (uint32_t)a.sbk;
  // per-lane offsets (the k-dependent part goes to the wave-uniform soffset); rows / columns past
  // M / N and k past the wave's range point past the descriptor and read 0 (address selects only)
  const uint32_t va = m0 + r < M ? 4u * ((uint32_t)(m0 + r) * lda + 4u * h) : a_bytes;
  const uint32_t vb = n0 + r < N ? (BKC ? 4u * ((uint32_t)(n0 + r) * ldb + 4u * h) : 4u * (4u * h * ldb + n0 + r))
                                 : b_bytes;
  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  auto load_set = [&](int sidx, floatx4 (&fa)[kDpU], floatx4 (&fb)[kDpU]) {
#pragma unroll
    for (int u = 0; u < kDpU; ++u) {
      const int k0 = kb + 8 * (sidx * kDpU + u);
      const bool kok = k0 + 4 * h < ke;
      fa[u] = bload4(ra, kok ? va : a_bytes, __builtin_amdgcn_readfirstlane(4u * (uint32_t)k0));
      if (BKC) {
        fb[u] = bload4(rb, kok ? vb : b_bytes, __builtin_amdgcn_readfirstlane(4u * (uint32_t)k0));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          fb[u][j] = bload(rb, kok ? vb : b_bytes, __builtin_amdgcn_readfirstlane(4u * (uint32_t)(k0 + j) * ldb));
      }
    }
  };
  auto mma_set = [&](const floatx4 (&fa)[kDpU], const floatx4 (&fb)[kDpU]) {
#pragma unroll
    for (int u = 0; u < kDpU; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[u][j], fb[u][j], acc, 0, 0, 0);
  };
  constexpr int KS = 8 * kDpU;
  const int ns = ke > kb ? (ke - kb + KS - 1) / KS : 0;
  floatx4 fa0[kDpU], fb0[kDpU], fa1[kDpU], fb1[kDpU];
  if (ns > 0) load_set(0, fa0, fb0);
  // loads unconditional (a set past the range reads 0): conditional ones leave hipcc waiting for
  // every load at the loop head
  for (int g = 0; g < ns; g += 2) {
    load_set(g + 1, fa1, fb1);
    __builtin_amdgcn_sched_barrier(0);
    mma_set(fa0, fb0);
    if (g + 1 >= ns) break;
    load_set(g + 2, fa0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    mma_set(fa1, fb1);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) red[w * 1024 + i * 64 + lane] = acc[i];
  __syncthreads();
  // output (row, col) is register (row & 3) + 4 (row >> 3) of lane col + 32 ((row >> 2) & 1)
  const int ri = (er & 3) + 4 * (er >> 3), rl = ec + 32 * ((er >> 2) & 1);
  float v[NO];
#pragma unroll
  for (int e = 0; e < NO; ++e) v[e] = 0.f;
#pragma unroll
  for (int u = 0; u < NW; ++u)
#pragma unroll
    for (int e = 0; e < NO; ++e) v[e] += red[u * 1024 + ri * 64 + rl + e];
  EpiPre<NO> epi;  // epi_load's arithmetic, term by term
  const float scale = a.drop_p < 1.f ? 1.f / (1.f - a.drop_p) : 0.f;
#pragma unroll
  for (int e = 0; e < NO; ++e) {
    float add = 0.f;
    if (a.beta != 0.f) add += a.beta * ec_c[e];
    if (a.bias) add += ec_b[e];
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (a.res[q]) add += ec_r[q][e];
    float dg = a.dact_pre ? act_grad(a.dact_kind, ec_p[e]) : 1.f;
    if (a.mask_in) dg *= ec_k[e] ? scale : 0.f;
    epi.add[e] = add;
    epi.dg[e] = dg;
  }
  epi_apply<NO>(a, em, en, v, epi);
}

struct Plan {
  int bm, bn, splits;
  int64_t kchunk;
  bool wgrad;
};

// Weight-gradient layout (A m-contiguous, B n-contiguous) with a long K: k_wgrad.
inline bool is_wgrad(const AimxGemmArgs& a) {
  // (also under AIMX_PREC_BF16: long-K weight gradients stay exact fp32 on k_wgrad — the tiled
  // kernel at these shapes, ~150 workgroups, measured 3-5x slower: profiles/r02_c4_amp_seq.txt)
  return a.sam == 1 && a.sbn == 1 && a.sak != 1 && a.K >= 512;
}

Plan plan_gemm(const AimxGemmArgs& a) {
  Plan p;
  p.wgrad = false;
  if (is_wgrad(a)) {
    // ~1536 waves in flight chip-wide, every wave keeping >= 2 load groups (2 x 32 k) of work
    p.wgrad = true;
    p.bm = p.bn = 32;
    const int64_t t = cdiv(a.M, 32) * cdiv(a.N, 32);
    // ~1150 workgroups (round 5, c2's 256 x 257 x 9170 concat dW: 6 splits 32.7 us, 16 splits
    // 27.1 us; the 76 x 77 ones 17.8 -> 15.9 us; profiles/r05_lone_wgrad_splits.txt)
    static const int64_t target = std::max<int64_t>(64, tune_i64("AIMX_WGRAD_WGS", 1152));
    int64_t splits = a.splits > 0 ? a.splits : cdiv(target, t);
    splits = std::max<int64_t>(1, std::min<int64_t>({splits, 64, a.K / 256}));
    p.kchunk = cdiv(cdiv(a.K, splits), 16) * 16;
    p.splits = (int)std::max<int64_t>(1, cdiv(a.K, p.kchunk));
    return p;
  }
  auto tiles = [&](int bm, int bn) { return cdiv(a.M, bm) * cdiv(a.N, bn); };
  // Pick the tile that minimises the busiest CU's MFMA work, ceil(tiles / CUs) * BM * BN (edge
  // tiles count in full: N = 152 runs 5 x 32 columns rather than 3 x 64); ties go to the larger
  // tile (fewer operand re-reads).
  // Grids of >= 2 full 64x64 waves over the chip keep 64x64 (operand reuse wins there).
  const int cand[3][2] = {{64, 64}, {64, 32}, {32, 32}};
  int64_t best = -1;
  for (const auto& c : cand) {
    if (best >= 0 && tiles(64, 64) >= 512) break;
    const int64_t w = cdiv(tiles(c[0], c[1]), 256) * c[0] * c[1];
    if (best < 0 || w < best) {
      best = w;
      p.bm = c[0];
      p.bn = c[1];
    }
  }
  // Small products (M·N·K < 7.5e8, K < 1024: c1–c3's projections, M ≈ 9 k rows, N, K ≤ 304; c4's
  // node-update GEMMs and head) take 32 x 32
  // tiles: ~2300 workgroups instead of ~580 hide the latency of their fused epilogues (bias,
  // activation, pre-activation / mask stores, residuals) — measured in the c2 step every such GEMM
  // is 10-20 % faster and the step 0.848 -> 0.809 ms, c3 1.033 -> 0.992 ms, although the bare
  // GEMMs (tools/gemm_micro.py, no epilogue operands) run faster on 64 x 64; c4/c5's larger
  // products keep the rule above (32 x 32 there: c4 3.48 -> 3.53, c5 5.23 -> 5.42 ms;
  // profiles/r02_gemm_tile_ab.txt).
  // (bounded at 7.5e8 and K < 1024: c5's 10.4 k x 307 x 307 node-update GEMMs run faster on
  // 64 x 64, and K >= 1024 products (c5's head GEMMs) on 64 x 64 with split K — per-GEMM step
  // traces in profiles/r02_gemm_tile_ab.txt)
  if (a.M * a.N * a.K < (int64_t)750000000 && a.K < 1024) p.bm = p.bn = 32;
  // Few rows, deep K (c5's post-pool F = 1024 chain, 258 x 1024 x 1024, 16 launches per step): 32 x 32
  // tiles split to ~1700 workgroups beat 64 x 32 split 4 (forward 15.8 -> 13.6 us, input gradient
  // 16.4 -> 14.1 us; the 3 x 8 tile / split sweep in profiles/r05_head_gemm_sweep.txt)
  const bool deep_few = tiles(64, 32) < 256 && a.K >= 1024 && a.M <= 1024;
  if (deep_few) p.bm = p.bn = 32;
  const int64_t t = tiles(p.bm, p.bn);
  int64_t splits = a.splits;
  if (splits <= 0 && deep_few) {
    splits = std::max<int64_t>(1, std::min<int64_t>((1728 + t / 2) / t, a.K / (4 * kBK)));
  } else if (splits <= 0) {
    splits = 1;
    // Split K only for grids short of one block per CU with a long K (weight gradients: K =
    // atoms; c5's head GEMMs: 264 x 1024 x 1024 ran as 160 64 x 32 blocks of 32 BK steps each, ~35
    // us, latency-bound), to ~512 blocks with every slice keeping >= 4 BK steps.
    if (t < 256 && a.K >= 1024) splits = std::min<int64_t>(cdiv(512, t), a.K / (4 * kBK));
  }
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, 64));
  p.kchunk = cdiv(cdiv(a.K, splits), kBK) * kBK;
  p.splits = (int)std::max<int64_t>(1, cdiv(a.K, p.kchunk));
  return p;
}

// 16-byte staging is legal when each operand's contiguous extent is a multiple of 4 floats and
// every row starts 16-byte aligned.
bool v4_ok(const AimxGemmArgs& a) {
  const bool ak = (a.sak == 1), bk = (a.sbk == 1);
  const int64_t Nreal = a.ones_col ? a.N - 1 : a.N;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al(a.A) || !al(a.B) || a.K % 4) return false;
  if (ak ? (a.sam % 4) : (a.sak % 4 || a.M % 4)) return false;
  if (bk ? (a.sbn % 4) : (a.sbk % 4 || Nreal % 4)) return false;
  return true;
}

template <int BM, int BN, bool V4, bool BF>
void launch_tile_v(const AimxGemmArgs& a, const Plan& p, dim3 grid, hipStream_t s, uint32_t ab, uint32_t bb) {
  const bool ak = (a.sak == 1), bk = (a.sbk == 1);
  const int kc = (int)p.kchunk;
  if (ak && bk)
    hipLaunchKernelGGL((k_gemm<BM, BN, true, true, V4, BF>), grid, dim3(256), 0, s, a, kc, ab, bb);
  else if (ak)
    hipLaunchKernelGGL((k_gemm<BM, BN, true, false, V4, BF>), grid, dim3(256), 0, s, a, kc, ab, bb);
  else if (bk)
    hipLaunchKernelGGL((k_gemm<BM, BN, false, true, V4, BF>), grid, dim3(256), 0, s, a, kc, ab, bb);
  else
    hipLaunchKernelGGL((k_gemm<BM, BN, false, false, V4, BF>), grid, dim3(256), 0, s, a, kc, ab, bb);
}

template <int BM, int BN>
void launch_tile(const AimxGemmArgs& a, const Plan& p, dim3 grid, hipStream_t s, uint32_t ab, uint32_t bb) {
  const bool bf = a.precision == AIMX_PREC_BF16;
  if (v4_ok(a)) {
    if (bf)
      launch_tile_v<BM, BN, true, true>(a, p, grid, s, ab, bb);
    else
      launch_tile_v<BM, BN, true, false>(a, p, grid, s, ab, bb);
  } else {
    if (bf)
      launch_tile_v<BM, BN, false, true>(a, p, grid, s, ab, bb);
    else
      launch_tile_v<BM, BN, false, false>(a, p, grid, s, ab, bb);
  }
}

}  // namespace

int wgrad_grouped_run(const AimxWgradProblem* p, int32_t n, void* workspace, size_t workspace_bytes,
                      int32_t* counters, int64_t n_counters, hipStream_t stream, int64_t min_wgs);
constexpr int64_t kLoneWgs = 1024;  // workgroups a lone long-K GEMM's LDS launch aims for

namespace {
struct WgPlan {
  int tiles_x, tiles_y, splits, kchunk;
  bool lds;    // k_wgrad_lds (bb x bb blocks) instead of k_wgrad_grouped (32 x 32 tiles)
  int bb;      // k_wgrad_lds block edge: 64 or 80 (wg_bb)
  int64_t slab;  // floats per split-K slab
};
// min_wgs > 0 (a lone long-K GEMM routed here): split K further until the launch has about that
// many workgroups, so the LDS fills of a few blocks are spread over the whole chip
// Block edge of one k_wgrad_lds launch: 64 (4 waves, one per SIMD: no SIMD carries two of a
// workgroup's waves into every fill barrier; with 80-wide blocks' 5 waves the barrier took 23-26 %
// of a wave's loop, tools/wgrad_trace.py) unless the 64-wide tiling pads the launch's long-K
// problems to more than 1.25x the block area of 80-wide blocks (c2's 76-wide MLP weights: 2.6x).
// Measured: c4 2.745 -> 2.635 ms, c5 4.025 -> 3.951 ms with 64; c2 0.722 -> 0.737 ms (kept at 80).
// The test hook AIMX_WGRAD_BB (aimx_set_option) forces 64 or 80.
int wg_bb(const AimxWgradProblem* p, int32_t n) {
  const int64_t force = opt_i64("AIMX_WGRAD_BB", 0);  // test hook (aimx_set_option): 64 or 80 forced
  if (force == 64 || force == 80) return (int)force;
  double a64 = 0, a80 = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (p[i].K < 2048) continue;
    const int64_t N = p[i].col_out ? p[i].N + 1 : p[i].N;
    a64 += (double)cdiv(p[i].M, 64) * cdiv(N, 64) * 64 * 64;
    a80 += (double)cdiv(p[i].M, 80) * cdiv(N, 80) * 80 * 80;
  }
  return a64 <= 1.25 * a80 ? 64 : 80;
}

WgPlan wg_plan(const AimxWgradProblem& p, int64_t min_wgs, int bb) {
  WgPlan w;
  const int64_t N = p.col_out ? p.N + 1 : p.N;
  if (p.K >= 2048) {
    // ~512 atoms of K per workgroup (16 LDS fills; ~2 workgroups per CU at c2's 36 blocks), 1024 for
    // problems of >= 9 blocks (c4 / c5: half the split-K slabs, longer fill pipelines — steps c4
    // 2.390 -> 2.376, c5 3.524 -> 3.502 ms; c2 keeps 512: 256 measured 0.717 vs 0.702;
    // profiles/r06_wgrad_kper_ab.txt)
    // (160-wide blocks measured slower: wgrad launch c4 472 -> 490 us, c5 853 -> 880 us, a quarter
    // of the workgroups at 109 VGPRs; profiles/r03_gemm_ab.txt — removed in round 6)
    w.lds = true;
    w.bb = bb;  // wg_bb
    w.slab = (int64_t)w.bb * w.bb;
    w.tiles_x = (int)cdiv(p.M, w.bb);
    w.tiles_y = (int)cdiv(N, w.bb);
    const int64_t kper =
        std::max<int64_t>(64, tune_i64("AIMX_WGRAD_KPER", (int64_t)w.tiles_x * w.tiles_y >= 9 ? 1024 : 512));
    int64_t sp = std::max<int64_t>(1, std::min<int64_t>(64, p.K / kper));
    if (min_wgs > 0)
      sp = std::max(sp, std::min<int64_t>({64, p.K / 128, cdiv(min_wgs, (int64_t)w.tiles_x * w.tiles_y)}));
    w.kchunk = (int)(cdiv(cdiv(p.K, sp), kWbK) * kWbK);
    // one split's rows of either operand under 2 GiB (its descriptors start at its first row): a
    // very long K (a large inference-time batch) takes more splits instead of a refusal
    const int64_t ld = std::max(p.ld_dy, p.ld_x), rows_max = ((1ll << 31) / 4 - 2 * ld) / ld;
    if (w.kchunk > rows_max) w.kchunk = (int)std::max<int64_t>(kWbK, rows_max / kWbK * kWbK);
    w.splits = (int)std::max<int64_t>(1, cdiv(p.K, w.kchunk));
    return w;
  }
  w.lds = false;
  w.bb = 0;
  w.slab = 1024;
  w.tiles_x = (int)cdiv(p.M, 32);
  w.tiles_y = (int)cdiv(N, 32);
  // ~1k atoms of K per workgroup: enough MFMA work per wave to amortise the fragment pipeline
  int64_t sp = std::max<int64_t>(1, std::min<int64_t>(64, p.K / 1024));
  w.kchunk = (int)(cdiv(cdiv(std::max<int64_t>(p.K, 1), sp), 16) * 16);
  w.splits = (int)std::max<int64_t>(1, cdiv(p.K, w.kchunk));
  return w;
}
bool wg_valid(const AimxWgradProblem& p) {
  if (p.M < 1 || p.N < 1 || p.K < 0 || !p.dY || !p.X || !p.dW) return false;
  if (p.ld_dy < p.M || p.ld_x < p.N || p.ld_dw < p.N) return false;
  if (p.zc_rowptr && (p.zc_chunks < 0 || p.zc_rows < 0 || p.zc_width < 0)) return false;
  if (p.K >= (1ll << 31) || p.M >= (1ll << 31) || p.N >= (1ll << 31)) return false;
  // the LDS-block kernel addresses each split from its first row (wg_plan bounds a split's rows);
  // the short-K kernel addresses the whole operand
  if (p.K >= 2048) return 4 * 64 * std::max(p.ld_dy, p.ld_x) < (1ll << 31);
  const int64_t a_ext = 4 * ((p.K - 1) * p.ld_dy + p.M), b_ext = 4 * ((p.K - 1) * p.ld_x + p.N);
  return p.K == 0 || (a_ext < (1ll << 31) && b_ext < (1ll << 31));
}

// A long-K weight-gradient GEMM with a plain-store epilogue (dW = dY^T X [+ ones-column bias
// gradient], optional zc_dim 1 trimming) runs as a one-problem k_wgrad_lds launch.
bool gemm_as_wgrad(const AimxGemmArgs& a, AimxWgradProblem& pr) {
  if (!(a.sam == 1 && a.sbn == 1 && a.sak != 1) || a.K < 1 || a.M < 1) return false;
  if (a.beta != 0.f || a.bias || a.res[0] || a.res[1] || a.res[2] || a.act_ncols > 0 || a.pre || a.dact_pre ||
      a.mask_in || a.mask_out || a.act >= 0)
    return false;
  if (a.zc_rowptr && a.zc_dim != 1) return false;
  // single long-K weight gradients: from M N K >= 2e9 (c4's 512-wide concat / embedding dW: step
  // 2.873 -> 2.836 ms; c2's 256-wide ones measured +72 us this way, c5's 1024-wide neutral);
  if ((double)a.M * (double)a.N * (double)a.K < 2e9) return false;
  pr = AimxWgradProblem{};
  pr.dY = a.A;
  pr.ld_dy = a.sak;
  pr.X = a.B;
  pr.ld_x = a.sbk;
  pr.dW = a.C;
  pr.ld_dw = a.ldc;
  pr.col_out = a.ones_col ? a.col_out : nullptr;
  pr.M = a.M;
  pr.N = a.ones_col ? a.N - 1 : a.N;
  pr.K = a.K;
  if (a.zc_rowptr) {
    pr.zc_rowptr = a.zc_rowptr;
    pr.zc_rows = a.zc_rows;
    pr.zc_chunks = a.zc_chunks;
    pr.zc_width = a.zc_width;
  }
  return pr.N >= 1 && wg_valid(pr) && wg_plan(pr, 0, 80).lds;
}
}  // namespace


// workspace of the tiled kernels' split-K plan
// k_gemm_deep: few rows, deep K (the post-pool chain at F >= 512: G x F x F, G <= 1024), A
// k-contiguous and B either way, 16-byte aligned k-contiguous rows, no ones column / trimming.
bool deep_ok(const AimxGemmArgs& a) {
  if (opt_i64("AIMX_GEMM_DEEP", 1) == 0 || a.precision != AIMX_PREC_FP32 || a.splits > 0) return false;
  if (a.ones_col || a.zc_rowptr || a.sak != 1 || (a.sbk != 1 && a.sbn != 1)) return false;
  if (a.M < 1 || a.M > 1024 || a.N < 1 || a.K < tune_i64("AIMX_GEMM_DEEP_KMIN", 512) || a.K % 4 != 0) return false;
  // enough tiles to spread over the CUs: the output layer (N = tasks: 8 tiles) is faster on the
  // split-K tiles (7.3 vs 13.4 us, profiles/r06_deep_gemm_micro.txt)
  const int64_t tiles = cdiv(a.M, 32) * cdiv(a.N, 32);
  if (tiles < 128 || tiles > 2048) return false;
  if (a.sam % 4 != 0 || (uintptr_t)a.A % 16 != 0) return false;
  if (a.sbk == 1 && (a.sbn % 4 != 0 || (uintptr_t)a.B % 16 != 0)) return false;
  // the epilogue operands' row extents (32-bit buffer offsets)
  const int64_t lds[6] = {a.ldc, a.ldres[0], a.ldres[1], a.ldres[2], a.lddact, a.ldmask};
  for (int64_t ld : lds)
    if (4 * ((a.M - 1) * std::max<int64_t>(ld, 0) + a.N) >= (1ll << 31)) return false;
  const int64_t a_ext = 4 * ((a.M - 1) * a.sam + a.K);
  const int64_t b_ext = a.sbk == 1 ? 4 * ((a.N - 1) * a.sbn + a.K) : 4 * ((a.K - 1) * a.sbk + a.N);
  return a_ext < (1ll << 31) && b_ext < (1ll << 31);
}

size_t tiled_workspace_floats(const AimxGemmArgs& a) {
  const Plan p = plan_gemm(a);
  return p.splits > 1 ? (size_t)p.splits * (size_t)(cdiv(a.M, p.bm) * cdiv(a.N, p.bn)) * p.bm * p.bn : 0;
}

// what the caller allocates: enough for whichever path launch_gemm takes (the k_wgrad_lds route
// needs counters, so a caller without them falls back to the tiled plan)
size_t gemm_workspace_floats(const AimxGemmArgs& a) {
  size_t f = tiled_workspace_floats(a);
  AimxWgradProblem pr;
  if (gemm_as_wgrad(a, pr)) {
    const WgPlan w = wg_plan(pr, kLoneWgs, wg_bb(&pr, 1));
    if (w.splits > 1) f = std::max(f, (size_t)w.splits * w.tiles_x * w.tiles_y * w.slab);
  }
  return f;
}

int launch_gemm(const AimxGemmArgs& a_in, hipStream_t s) {
  AimxGemmArgs a = a_in;
  if (a.M < 0 || a.N < 0 || a.K < 0) return AIMX_EARG;
  if (a.precision != AIMX_PREC_FP32 && a.precision != AIMX_PREC_BF16) return AIMX_EARG;
  if (a.M == 0 || a.N == 0) return AIMX_OK;
  if (a.ones_col && (!a.col_out || a.N < 1)) return AIMX_EARG;
  if ((a.mask_out || a.mask_in) && !(a.drop_p < 1.f)) return AIMX_EARG;
  if (a.mask_out && !a.drop_seed) return AIMX_EARG;
  if (a.zc_rowptr) {  // trimming: sane chunk geometry; zc_dim 1 / 2 only with a plain-store epilogue
    if (a.zc_chunks < 0 || a.zc_rows < 0 || a.zc_width < 0 || a.zc_dim < 0 || a.zc_dim > 2) return AIMX_EARG;
    if (a.zc_width * (a.zc_chunks + 1) >= (1ll << 31)) return AIMX_EARG;
    if (a.zc_dim != 0 && (a.beta != 0.f || a.bias || a.res[0] || a.res[1] || a.res[2] || a.act_ncols > 0 ||
                          a.pre || a.dact_pre || a.mask_in || a.mask_out))
      return AIMX_EARG;
  }
  {
    AimxWgradProblem pr;
    if (gemm_as_wgrad(a, pr)) {
      const WgPlan w = wg_plan(pr, kLoneWgs, wg_bb(&pr, 1));
      const size_t need = w.splits > 1 ? sizeof(float) * w.splits * w.tiles_x * w.tiles_y * w.slab : 0;
      if ((w.splits == 1 || (a.workspace && a.workspace_bytes >= need)) && a.counters &&
          (int64_t)w.tiles_x * w.tiles_y <= a.n_counters)
        return wgrad_grouped_run(&pr, 1, a.workspace, a.workspace_bytes, a.counters, a.n_counters, s, kLoneWgs);
    }
  }
  if (deep_ok(a)) {
    const int tm = (int)cdiv(a.M, 32), nt = tm * (int)cdiv(a.N, 32);
    // 16 waves (each 1/16 of K: c5's K = 1024 is two register sets per wave, all in flight at once);
    // 8 in the tuning build's A/B (AIMX_GEMM_DEEP=8)
    const int nw = opt_i64("AIMX_GEMM_DEEP", 16) == 8 ? 8 : 16;
    const int kq = (int)(cdiv(cdiv(a.K, nw), 8) * 8);
    const uint32_t a_bytes = (uint32_t)(4 * ((a.M - 1) * a.sam + a.K));
    const uint32_t b_bytes = (uint32_t)(a.sbk == 1 ? 4 * ((a.N - 1) * a.sbn + a.K) : 4 * ((a.K - 1) * a.sbk + a.N));
    using Fn = void (*)(const AimxGemmArgs, int, int, int, uint32_t, uint32_t);
    const Fn fn = a.sbk == 1 ? (nw == 16 ? k_gemm_deep<true, 16> : k_gemm_deep<true, 8>)
                             : (nw == 16 ? k_gemm_deep<false, 16> : k_gemm_deep<false, 8>);
    hipLaunchKernelGGL(fn, dim3((unsigned)nt), dim3(64 * nw), 0, s, a, tm, nt, kq, a_bytes, b_bytes);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  }
  // operand layouts: each operand must be contiguous along k or along m/n; byte extents < 2 GiB
  if (!(a.sak == 1 || a.sam == 1) || !(a.sbk == 1 || a.sbn == 1)) return AIMX_EARG;
  const int64_t Nreal = a.ones_col ? a.N - 1 : a.N;
  const int64_t a_ext = 4 * ((a.M - 1) * a.sam + (a.K - 1) * a.sak + 1);
  const int64_t b_ext = Nreal > 0 ? 4 * ((a.K - 1) * a.sbk + (Nreal - 1) * a.sbn + 1) : 4;
  if (a.K > 0 && a_ext >= (1ll << 31) && a.sak == 1 && a.M > 1) {
    // A's rows past 2 GiB (a very large batch: ~250 k atoms at c5's F-row stride): consecutive row
    // chunks of the product, each its own launch over offset row pointers (rows are independent;
    // the epilogue operands are row-indexed, the dropout hash keyed by the global row)
    const int64_t rows = std::max<int64_t>(1, ((1ll << 31) / 4 - a.K - 64) / std::max<int64_t>(a.sam, 1));
    for (int64_t m0 = 0; m0 < a.M; m0 += rows) {
      AimxGemmArgs c = a;
      c.M = std::min(rows, a.M - m0);
      c.m_base = a.m_base + m0;
      c.A = a.A + m0 * a.sam;
      c.C = a.C + m0 * a.ldc;
      if (a.pre) c.pre = a.pre + m0 * a.ldpre;
      if (a.dact_pre) c.dact_pre = a.dact_pre + m0 * a.lddact;
      for (int r = 0; r < 3; ++r)
        if (a.res[r]) c.res[r] = a.res[r] + m0 * a.ldres[r];
      if (a.mask_in) c.mask_in = a.mask_in + m0 * a.ldmask;
      if (a.mask_out) c.mask_out = a.mask_out + m0 * a.ldmask;
      if (a.col_out) c.col_out = a.col_out + m0;
      const int rc = launch_gemm(c, s);
      if (rc != AIMX_OK) return rc;
    }
    return AIMX_OK;
  }
  if (a.K > 0 && (a_ext >= (1ll << 31) || b_ext >= (1ll << 31))) return AIMX_EARG;
  if (a.M >= (1ll << 31) || a.N >= (1ll << 31) || a.K >= (1ll << 31)) return AIMX_EARG;
  // descriptor byte counts = the operand's true extent: every in-range element is readable, loads
  // past the end return 0; rows/columns beyond M/N that still fall inside the extent only feed
  // output rows/columns that are never stored, and k beyond the slice end is zeroed by a select
  const uint32_t a_bytes = (uint32_t)std::max<int64_t>(a_ext, 4);
  const uint32_t b_bytes = (uint32_t)std::max<int64_t>(b_ext, 4);
  Plan p = plan_gemm(a);
  if (p.splits > 1 && (!a.workspace || a.workspace_bytes < sizeof(float) * tiled_workspace_floats(a))) {
    p.splits = 1;
    p.kchunk = std::max<int64_t>(cdiv(a.K, kBK) * kBK, kBK);
  }
  if (p.splits == 1 && p.wgrad) p.kchunk = cdiv(a.K, 16) * 16;
  if (a.K == 0) p.splits = 1, p.kchunk = kBK;
  dim3 grid((unsigned)cdiv(a.M, p.bm), (unsigned)cdiv(a.N, p.bn), (unsigned)p.splits);
  if (p.splits > 1 && a.counters && (int64_t)grid.x * grid.y > a.n_counters) a.counters = nullptr;
  if (p.splits == 1) a.counters = nullptr;
  if (p.wgrad && a.K > 0)
    hipLaunchKernelGGL(k_wgrad, grid, dim3(256), 0, s, a, (int)p.kchunk, a_bytes, b_bytes);
  else if (p.bm == 64 && p.bn == 64)
    launch_tile<64, 64>(a, p, grid, s, a_bytes, b_bytes);
  else if (p.bm == 64)
    launch_tile<64, 32>(a, p, grid, s, a_bytes, b_bytes);
  else
    launch_tile<32, 32>(a, p, grid, s, a_bytes, b_bytes);
  AIMX_CHECK_LAUNCH();
  if (p.splits > 1 && !a.counters) {
    const int64_t blocks = std::min<int64_t>(cdiv(a.M * a.N, 256), 2048);
    const int tn = (int)grid.y;
    if (p.bm == 64 && p.bn == 64)
      hipLaunchKernelGGL((k_splitk_reduce<64, 64>), dim3((unsigned)blocks), dim3(256), 0, s, a, p.splits, tn);
    else if (p.bm == 64)
      hipLaunchKernelGGL((k_splitk_reduce<64, 32>), dim3((unsigned)blocks), dim3(256), 0, s, a, p.splits, tn);
    else
      hipLaunchKernelGGL((k_splitk_reduce<32, 32>), dim3((unsigned)blocks), dim3(256), 0, s, a, p.splits, tn);
    AIMX_CHECK_LAUNCH();
  }
  return AIMX_OK;
}

}  // namespace aimx


namespace aimx {
size_t wgrad_ws_bytes(const AimxWgradProblem* p, int32_t n, int64_t min_wgs) {
  if (!p || n < 0) return 0;
  size_t f = 0;
  const int bb = wg_bb(p, n);
  for (int32_t i = 0; i < n; ++i) {
    const WgPlan w = wg_plan(p[i], min_wgs, bb);
    if (w.splits > 1) f += (size_t)w.splits * w.tiles_x * w.tiles_y * w.slab;
  }
  return sizeof(float) * f;
}

int wgrad_grouped_run(const AimxWgradProblem* p, int32_t n, void* workspace, size_t workspace_bytes,
                      int32_t* counters, int64_t n_counters, hipStream_t stream, int64_t min_wgs) {
  if (!p || n < 0) return AIMX_EARG;
  for (int32_t i = 0; i < n; ++i)
    if (!wg_valid(p[i])) return AIMX_EARG;
  if (workspace_bytes < wgrad_ws_bytes(p, n, min_wgs) || (workspace_bytes && !workspace)) return AIMX_EARG;
  int64_t ctiles = 0;
  const int bb = wg_bb(p, n);
  for (int32_t i = 0; i < n; ++i) {
    const WgPlan w = wg_plan(p[i], min_wgs, bb);
    ctiles += (int64_t)w.tiles_x * w.tiles_y;
  }
  if (!counters || ctiles > n_counters) return AIMX_EARG;
  // long-K problems -> k_wgrad_lds launches, the rest -> k_wgrad_grouped launches (<= kWgMaxProb
  // problems per launch each); workspace slabs and counters are laid out in problem order
  int64_t ws_off = 0, cnt_off = 0;
  WgradTable t{};
  WbTable tb{};
  int32_t blk = 0, blkb = 0;
  auto flush = [&](bool lds) {
    if (lds) {
      tb.blk0[tb.n] = blkb;
      tb.xcd = 1;
      if (blkb > 0) {
        int nv4 = 0;
        for (int k = 0; k < tb.n; ++k) nv4 += tb.v4[k] != 0;
        const int vm = nv4 == tb.n ? 1 : (nv4 == 0 ? 0 : 2);
        using WbFn = void (*)(const WbTable, float*, int32_t*);
        WbFn fn;
        const bool narrow = bb == 64;
        // double-buffered LDS (0.5-1.5 % faster at c4 / c5, neutral at c2; profiles/r03_wgrad_dbuf_ab.txt)
        if (narrow)
          fn = vm == 1 ? k_wgrad_lds<64, 1> : (vm == 0 ? k_wgrad_lds<64, 0> : k_wgrad_lds<64, 2>);
        else
          fn = vm == 1 ? k_wgrad_lds<80, 1> : (vm == 0 ? k_wgrad_lds<80, 0> : k_wgrad_lds<80, 2>);
        const int nthr = narrow ? WbGeom<64>::T : WbGeom<80>::T;
        hipLaunchKernelGGL(fn, dim3((unsigned)blkb), dim3(nthr), 0, (hipStream_t)stream, tb, (float*)workspace, counters);
      }
      tb = WbTable{};
      blkb = 0;
    } else {
      t.blk0[t.n] = blk;
      if (blk > 0)
        hipLaunchKernelGGL(k_wgrad_grouped, dim3((unsigned)blk), dim3(256), 0, (hipStream_t)stream, t, (float*)workspace,
                           counters);
      t = WgradTable{};
      blk = 0;
    }
  };
  for (int32_t i = 0; i < n; ++i) {
    const AimxWgradProblem& pr = p[i];
    const WgPlan w = wg_plan(pr, min_wgs, bb);
    const int32_t nt = w.tiles_x * w.tiles_y;
    if (w.lds) {
      const int k = tb.n++;
      const int64_t Kr = std::max<int64_t>(pr.K, 1) - 1;
      const bool v4 = pr.ld_dy % 4 == 0 && pr.ld_x % 4 == 0 && (uintptr_t)pr.dY % 16 == 0 && (uintptr_t)pr.X % 16 == 0;
      tb.p[k] = pr;
      tb.blk0[k] = blkb;
      tb.bn[k] = w.tiles_y;
      tb.nblk[k] = nt;
      tb.splits[k] = w.splits;
      tb.kchunk[k] = w.kchunk;
      tb.v4[k] = v4;
      // a float4 straddling the last row's edge stays inside the descriptor (rows are ld >= the
      // rounded width long), so its valid components are never cut by the range check
      const int64_t am = v4 ? std::min<int64_t>(pr.ld_dy, cdiv(pr.M, 4) * 4) : pr.M;
      const int64_t bm = v4 ? std::min<int64_t>(pr.ld_x, cdiv(pr.N, 4) * 4) : pr.N;
      const int64_t Ks = std::min<int64_t>(Kr, w.kchunk - 1);  // rows of one split past its first
      tb.a_bytes[k] = (uint32_t)std::max<int64_t>(4, 4 * (Ks * pr.ld_dy + am));
      tb.b_bytes[k] = (uint32_t)std::max<int64_t>(4, 4 * (Ks * pr.ld_x + bm));
      tb.ws_off[k] = ws_off;
      tb.cnt_off[k] = cnt_off;
      blkb += w.splits * nt;
      if (tb.n == kWgMaxProb) flush(true);
    } else {
      const int k = t.n++;
      t.p[k] = pr;
      t.blk0[k] = blk;
      t.tiles_y[k] = w.tiles_y;
      t.ntiles[k] = nt;
      t.splits[k] = w.splits;
      t.kchunk[k] = w.kchunk;
      t.a_bytes[k] = (uint32_t)std::max<int64_t>(4, 4 * ((std::max<int64_t>(pr.K, 1) - 1) * pr.ld_dy + pr.M));
      t.b_bytes[k] = (uint32_t)std::max<int64_t>(4, 4 * ((std::max<int64_t>(pr.K, 1) - 1) * pr.ld_x + pr.N));
      t.ws_off[k] = ws_off;
      t.cnt_off[k] = cnt_off;
      blk += w.splits * nt;
      if (t.n == kWgMaxProb) flush(false);
    }
    if (w.splits > 1) ws_off += (int64_t)w.splits * nt * w.slab;
    cnt_off += nt;
  }
  if (t.n) flush(false);
  if (tb.n) flush(true);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
}  // namespace aimx

extern "C" size_t aimx_wgrad_grouped_workspace_bytes(const AimxWgradProblem* p, int32_t n) {
  return aimx::wgrad_ws_bytes(p, n, 0);
}

extern "C" int aimx_wgrad_grouped(const AimxWgradProblem* p, int32_t n, void* workspace, size_t workspace_bytes,
                                  int32_t* counters, int64_t n_counters, aimx_stream_t stream) {
  return aimx::wgrad_grouped_run(p, n, workspace, workspace_bytes, counters, n_counters, (hipStream_t)stream, 0);
}

extern "C" size_t aimx_gemm_workspace_bytes(const AimxGemmArgs* a) {
  return a ? sizeof(float) * aimx::gemm_workspace_floats(*a) : 0;
}

extern "C" int aimx_gemm(const AimxGemmArgs* a, aimx_stream_t stream) {
  if (!a) return AIMX_EARG;
  return aimx::launch_gemm(*a, (hipStream_t)stream);
}

#ifdef AIMX_WB_TRACE
extern "C" int aimx_wb_trace_read(long long* out) {  // 4 x 10 x 5 shader-clock totals
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(aimx::g_wb_trace), sizeof(long long) * 4 * 10 * 5) == hipSuccess ? 0 : -1;
}
#endif
