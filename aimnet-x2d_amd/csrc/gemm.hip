// Fused fp32 GEMM on CDNA4 matrix cores for the node-update MLP.
//
// Reference: ShellConvolutionLayer.forward, src/models/layers.py:82-106 (nn.Linear = addmm,
// SiLU, Dropout, residual adds) and its autograd backward. Every contraction there is fp32, so
// the MFMA is v_mfma_f32_16x16x4_f32: exact f32 products accumulated as a k-ordered fmaf chain,
// at the f32 matrix rate (64 FLOP/clk/SIMD, ~157 TF/s chip). There is no xf32 path on gfx950.
//
// Tiling: 256 threads = 4 waves in a 2x2 grid over a BM x BN block tile, each wave owning a
// (BM/2) x (BN/2) sub-tile as (BM/32) x (BN/32) 16x16 accumulators. K advances in BK = 16
// slices staged in LDS as k-major [BK][BM+16] / [BK][BN+16] images (row stride = 16 mod 32 banks
// so the two k rows a 32-lane group reads land on disjoint banks). The next slice is prefetched
// into registers while the MFMAs of the current slice run. The staging loop picks the
// coalesced direction from the operand strides (row- or column-major, both occur: Y = X W^T
// forward, dX = dY W and dW = dY^T X backward).
// Epilogue (fused, see include/aimx.h): bias, residuals, pre-activation store, activation,
// hash-dropout with mask store, mask/act' multiplication for the backward, and an implicit ones
// column that turns the weight-gradient GEMM's last column into the bias gradient.
// Long-K / small-MN products (weight gradients, K = atoms) run split-K with fp32 partial slabs
// and an ordered reduce: deterministic, no atomics.
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kBK = 16;

__device__ __forceinline__ void epilogue(const AimxGemmArgs& a, int64_t m, int64_t n, float v) {
  if (a.ones_col && n == a.N - 1) {
    a.col_out[m] = v;
    return;
  }
  float* cp = a.C + m * a.ldc + n;
  if (a.beta != 0.f) v += a.beta * *cp;
  if (a.bias) v += a.bias[n];
#pragma unroll
  for (int r = 0; r < 3; ++r)
    if (a.res[r]) v += a.res[r][m * a.ldres[r] + n];
  if (n < a.act_ncols) {
    if (a.pre) a.pre[m * a.ldpre + n] = v;
    if (a.act >= 0) v = act_fwd(a.act, v);
  }
  if (a.mask_out) {
    const float scale = 1.f / (1.f - a.drop_p);
    const bool keep = hash_uniform((uint64_t)*a.drop_seed, a.drop_salt, (uint64_t)m * (uint64_t)a.N + (uint64_t)n) >= a.drop_p;
    v = keep ? v * scale : 0.f;
    a.mask_out[m * a.ldmask + n] = keep ? 1 : 0;
  }
  if (a.mask_in) {
    const float scale = 1.f / (1.f - a.drop_p);
    v = a.mask_in[m * a.ldmask + n] ? v * scale : 0.f;
  }
  if (a.dact_pre) v *= act_grad(a.dact_kind, a.dact_pre[m * a.lddact + n]);
  *cp = v;
}

template <int BM, int BN>
__global__ __launch_bounds__(256) void k_gemm(const AimxGemmArgs a, int64_t kchunk) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int SA = BM + 16, SB = BN + 16;
  constexpr int NA = BM * kBK / 256, NB = BN * kBK / 256;  // staged elements per thread
  __shared__ float As[kBK * SA];
  __shared__ float Bs[kBK * SB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * kchunk;
  const int64_t kend = min(a.K, kbeg + kchunk);
  const bool a_mfast = (a.sam == 1 && a.sak != 1);
  const bool b_nfast = (a.sbn == 1 && a.sbk != 1);
  const int64_t Nreal = a.ones_col ? a.N - 1 : a.N;

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  float ra[NA], rb[NB];
  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + i * 256;
      const int mm = a_mfast ? (idx % BM) : (idx / kBK);
      const int kk = a_mfast ? (idx / BM) : (idx % kBK);
      const int64_t m = m0 + mm, k = k0 + kk;
      ra[i] = (m < a.M && k < kend) ? a.A[m * a.sam + k * a.sak] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + i * 256;
      const int nn = b_nfast ? (idx % BN) : (idx / kBK);
      const int kk = b_nfast ? (idx / BN) : (idx % kBK);
      const int64_t n = n0 + nn, k = k0 + kk;
      float v = 0.f;
      if (k < kend) {
        if (n < Nreal)
          v = a.B[k * a.sbk + n * a.sbn];
        else if (a.ones_col && n == a.N - 1)
          v = 1.f;
      }
      rb[i] = v;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + i * 256;
      const int mm = a_mfast ? (idx % BM) : (idx / kBK);
      const int kk = a_mfast ? (idx / BM) : (idx % kBK);
      As[kk * SA + mm] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + i * 256;
      const int nn = b_nfast ? (idx % BN) : (idx / kBK);
      const int kk = b_nfast ? (idx / BN) : (idx % kBK);
      Bs[kk * SB + nn] = rb[i];
    }
  };

  if (kbeg < kend) load_tile(kbeg);
  for (int64_t k0 = kbeg; k0 < kend; k0 += kBK) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (k0 + kBK < kend) load_tile(k0 + kBK);
#pragma unroll
    for (int s = 0; s < kBK / 4; ++s) {
      const int kr = 4 * s + (lane >> 4);
      float af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = As[kr * SA + wr * WM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = Bs[kr * SB + wc * WN + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }

  // C/D layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg.
  const bool partial = gridDim.z > 1;
  float* ws = a.workspace + (int64_t)blockIdx.z * a.M * a.N;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wr * WM + i * 16 + (lane >> 4) * 4 + r;
        const int64_t n = n0 + wc * WN + j * 16 + (lane & 15);
        if (m < a.M && n < a.N) {
          if (partial)
            ws[m * a.N + n] = acc[i][j][r];
          else
            epilogue(a, m, n, acc[i][j][r]);
        }
      }
}

__global__ void k_splitk_reduce(const AimxGemmArgs a, int splits) {
  const int64_t total = a.M * a.N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += a.workspace[(int64_t)z * total + t];
    epilogue(a, t / a.N, t % a.N, v);
  }
}

struct Plan {
  int bm, bn, splits;
  int64_t kchunk;
};

Plan plan_gemm(const AimxGemmArgs& a) {
  Plan p;
  p.bm = 64;
  p.bn = a.N <= 32 ? 32 : 64;
  const int64_t tiles = cdiv(a.M, p.bm) * cdiv(a.N, p.bn);
  int64_t splits = a.splits;
  if (splits <= 0) {
    splits = 1;
    if (tiles < 192 && a.K >= 512) splits = std::min<int64_t>(cdiv(384, tiles), a.K / 256);
  }
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, 64));
  p.kchunk = cdiv(cdiv(a.K, splits), kBK) * kBK;
  p.splits = (int)cdiv(a.K, p.kchunk);
  if (p.splits < 1) p.splits = 1;
  return p;
}

}  // namespace

size_t gemm_workspace_floats(const AimxGemmArgs& a) {
  const Plan p = plan_gemm(a);
  return p.splits > 1 ? (size_t)p.splits * (size_t)a.M * (size_t)a.N : 0;
}

int launch_gemm(const AimxGemmArgs& a_in, hipStream_t s) {
  AimxGemmArgs a = a_in;
  if (a.M < 0 || a.N < 0 || a.K < 0) return AIMX_EARG;
  if (a.M == 0 || a.N == 0) return AIMX_OK;
  if (a.ones_col && (!a.col_out || a.N < 1)) return AIMX_EARG;
  if ((a.mask_out || a.mask_in) && !(a.drop_p < 1.f)) return AIMX_EARG;
  if (a.mask_out && !a.drop_seed) return AIMX_EARG;
  Plan p = plan_gemm(a);
  if (p.splits > 1 && (!a.workspace || a.workspace_bytes < sizeof(float) * (size_t)p.splits * a.M * a.N)) {
    p.splits = 1;
    p.kchunk = std::max<int64_t>(cdiv(a.K, kBK) * kBK, kBK);
  }
  if (a.K == 0) p.splits = 1, p.kchunk = kBK;
  dim3 grid((unsigned)cdiv(a.M, p.bm), (unsigned)cdiv(a.N, p.bn), (unsigned)p.splits);
  if (p.bn == 32)
    hipLaunchKernelGGL((k_gemm<64, 32>), grid, dim3(256), 0, s, a, p.kchunk);
  else
    hipLaunchKernelGGL((k_gemm<64, 64>), grid, dim3(256), 0, s, a, p.kchunk);
  AIMX_CHECK_LAUNCH();
  if (p.splits > 1) {
    const int64_t blocks = std::min<int64_t>(cdiv(a.M * a.N, 256), 2048);
    hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)blocks), dim3(256), 0, s, a, p.splits);
    AIMX_CHECK_LAUNCH();
  }
  return AIMX_OK;
}

}  // namespace aimx

extern "C" size_t aimx_gemm_workspace_bytes(const AimxGemmArgs* a) {
  return a ? sizeof(float) * aimx::gemm_workspace_floats(*a) : 0;
}

extern "C" int aimx_gemm(const AimxGemmArgs* a, aimx_stream_t stream) {
  if (!a) return AIMX_EARG;
  return aimx::launch_gemm(*a, (hipStream_t)stream);
}
