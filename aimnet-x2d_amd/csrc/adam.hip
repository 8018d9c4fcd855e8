// Fused global-norm gradient clipping + Adam over a list of tensors (two launches per step).
//
// Reference: the trainer's step, src/training/trainer.py:163-164
//   torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0); optimizer.step()
// with optimizer = torch.optim.Adam(model.parameters(), lr) (trainer.py:221-223). PyTorch runs
// these as ~2 elementwise launches per parameter tensor (plus foreach norm kernels): hundreds of
// 3-5 us launches per step for this model. Here:
//   1. k_adam_sumsq   : per-(tensor, slice) partial sums of g^2 (fp64)  -> workspace
// (each tensor's own step counter, torch.optim.Adam's per-parameter state['step'], is advanced by
// the first workgroup of that tensor in launch 1 and read by launch 2 for its bias corrections:
// a parameter without a gradient in a step keeps its count, as in torch)
//   2. k_adam_update  : every workgroup first folds the partials in one fixed order (total norm,
//                       clip coefficient: deterministic, no arrival atomics, the same bits in every
//                       workgroup), then g *= coef (in place, as clip_grad_norm_ leaves it), [g += wd * p],
//                       m = lerp(m, g, 1 - beta1), v = beta2 v + (1 - beta2) g^2,
//                       p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// The tensor table travels in the kernel arguments (chunks of kAdamChunk tensors), so nothing is
// copied host->device and the two launches capture into a HIP graph as plain kernel nodes. The
// sum-of-squares slice (one workgroup) is 2048 elements or more, sized so a call makes about
// kTargetSlices partials (c5's ~15M parameters: 16384-element slices, ~1,000 partials instead of
// 7,284, each of which used to end in an atomic arrival on one counter: a serialised ~80 us tail);
// the update keeps 2048-element slices (many workgroups: it moves 8 bytes per byte the sum reads). The
// step counter and the per-group learning rates live in device memory (capturable).
#include <algorithm>
#include <cmath>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kAdamChunk = 80;        // tensors per launch (kernel-argument table, < 4 KiB: a
                                      // reference GNN's ~75 parameters take one launch each way)
constexpr int kAdamThreads = 256;
constexpr int64_t kSliceElems = 2048; // smallest workgroup slice (8 elements per thread)
constexpr int64_t kTargetSlices = 1536;  // about this many slices per call (>> 256 CUs)

struct AdamTable {
  int32_t n;
  int32_t blk0[kAdamChunk + 1];  // first workgroup of each tensor (relative to the chunk)
  int32_t gs[kAdamChunk];        // parameter group | step slot << 8
  int64_t numel[kAdamChunk];
  float* param[kAdamChunk];
  float* grad[kAdamChunk];
  float* m[kAdamChunk];
  float* v[kAdamChunk];
};
static_assert(sizeof(AdamTable) <= 4000, "kernel argument table must stay under the 4 KiB limit");

__device__ __forceinline__ int find_tensor(const AdamTable& t, int b) {
  int i = 0;
  while (i + 1 < t.n && t.blk0[i + 1] <= b) ++i;
  return i;
}

// The clip coefficient from every slice's partial sum of squares, by one workgroup: thread t sums
// partials t, t + 256, ... in that order with 8 loads in flight, then the threads' sums are
// combined in a fixed order. Deterministic: the same bits every call and in every workgroup that
// runs it — the update's workgroups each fold the partials themselves (round 5: one launch fewer
// per step; the partials are ~0.5-1k doubles, L2-resident). Returns (coef, total norm).
__device__ __forceinline__ float2 fold_partials(const double* __restrict__ partial, int64_t n_partial, float max_norm,
                                                double* red) {
  constexpr int kInFlight = 8;
  double s = 0.0;
  for (int64_t j0 = threadIdx.x; j0 < n_partial; j0 += (int64_t)kInFlight * kAdamThreads) {
    double v[kInFlight];
#pragma unroll
    for (int q = 0; q < kInFlight; ++q) {
      const int64_t j = j0 + (int64_t)q * kAdamThreads;
      v[q] = j < n_partial ? partial[j] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kInFlight; ++q) s += v[q];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < kAdamThreads / kWave; ++w) t += red[w];
  const float total = (float)sqrt(t);
  float coef = 1.f;
  if (max_norm > 0.f) coef = fminf(max_norm / (total + 1e-6f), 1.f);
  return make_float2(coef, total);
}

// Launch 1: the partial sum of squares of each slice (fp64; the first workgroup of each tensor
// advances that tensor's step counter).
__global__ __launch_bounds__(kAdamThreads) void k_adam_sumsq(const AdamTable t, double* __restrict__ partial,
                                                             float* __restrict__ steps, int64_t base,
                                                             int64_t slice) {
  const int i = find_tensor(t, blockIdx.x);
  if (blockIdx.x == t.blk0[i] && threadIdx.x == 0) steps[t.gs[i] >> 8] += 1.f;
  const int64_t s0 = (int64_t)(blockIdx.x - t.blk0[i]) * slice;
  const int64_t s1 = min(t.numel[i], s0 + slice);
  const float* __restrict__ g = t.grad[i];
  double acc = 0.0;
  int64_t j0 = s0;
  if ((((uintptr_t)g) & 15) == 0) {  // 16-byte loads (same fp64 sums, per-thread order changes)
    const int64_t q1 = s0 + ((s1 - s0) & ~(int64_t)3);
#pragma unroll 4
    for (int64_t j = s0 + 4 * threadIdx.x; j < q1; j += 4 * kAdamThreads) {
      const floatx4 x = *reinterpret_cast<const floatx4*>(g + j);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += (double)x[e] * (double)x[e];
    }
    j0 = q1;
  }
#pragma unroll 8
  for (int64_t j = j0 + threadIdx.x; j < s1; j += kAdamThreads) {
    const double x = g[j];
    acc += x * x;
  }
  __shared__ double red[kAdamThreads / kWave];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < kAdamThreads / kWave; ++w) s += red[w];
    partial[base + blockIdx.x] = s;
  }
}

// Launch 2.
// scal[0] = clip coefficient, scal[3] = total gradient norm (the value clip_grad_norm_ returns),
// written by the first launch's workgroup 0
__global__ __launch_bounds__(kAdamThreads) void k_adam_update(const AdamTable t, const double* __restrict__ partial,
                                                              int64_t n_partial, float max_norm, float* __restrict__ scal,
                                                              float* __restrict__ norm_out, int32_t first,
                                                              int64_t slice, const float* __restrict__ steps,
                                                              const float* __restrict__ lr, float beta1, float omb1,
                                                              float beta2, float omb2, float eps, float wd) {
  __shared__ double red[kAdamThreads / kWave];
  const float2 cn = fold_partials(partial, n_partial, max_norm, red);
  const float coef = cn.x;
  if (first && blockIdx.x == 0 && threadIdx.x == 0) {
    scal[0] = coef;
    scal[3] = cn.y;
    if (norm_out) *norm_out = cn.y;
  }
  const int i = find_tensor(t, blockIdx.x);
  const int64_t s0 = (int64_t)(blockIdx.x - t.blk0[i]) * slice;
  const int64_t s1 = min(t.numel[i], s0 + slice);
  const float st = steps[t.gs[i] >> 8];
  const float inv_bc1 = 1.f / (1.f - powf(beta1, st)), bc2s = sqrtf(1.f - powf(beta2, st));
  const float step_size = lr[t.gs[i] & 255] * inv_bc1;
  float* __restrict__ p = t.param[i];
  float* __restrict__ g = t.grad[i];
  float* __restrict__ m = t.m[i];
  float* __restrict__ v = t.v[i];
  auto upd = [&](float& gj_io, float& pj_io, float& mj_io, float& vj_io) {
    float gj = gj_io * coef;
    gj_io = gj;
    const float pj = pj_io;
    if (wd != 0.f) gj += wd * pj;
    const float mj = mj_io + omb1 * (gj - mj_io);     // exp_avg.lerp_(grad, 1 - beta1)
    const float vj = beta2 * vj_io + omb2 * gj * gj;  // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
    mj_io = mj;
    vj_io = vj;
    pj_io = pj - step_size * (mj / (sqrtf(vj) / bc2s + eps));
  };
  // 16-byte accesses when all four tensors are 16-byte aligned (a dword access moves a quarter
  // of the bytes per address cycle); the same per-element arithmetic, so results are unchanged
  const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0;
  int64_t j0 = s0;
  if (vec) {
    const int64_t q1 = s0 + ((s1 - s0) & ~(int64_t)3);
#pragma unroll 2
    for (int64_t j = s0 + 4 * threadIdx.x; j < q1; j += 4 * kAdamThreads) {
      floatx4 gv = *reinterpret_cast<const floatx4*>(g + j), pv = *reinterpret_cast<const floatx4*>(p + j);
      floatx4 mv = *reinterpret_cast<const floatx4*>(m + j), vv = *reinterpret_cast<const floatx4*>(v + j);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float ge = gv[e], pe = pv[e], me = mv[e], ve = vv[e];
        upd(ge, pe, me, ve);
        gv[e] = ge;
        pv[e] = pe;
        mv[e] = me;
        vv[e] = ve;
      }
      *reinterpret_cast<floatx4*>(g + j) = gv;
      *reinterpret_cast<floatx4*>(p + j) = pv;
      *reinterpret_cast<floatx4*>(m + j) = mv;
      *reinterpret_cast<floatx4*>(v + j) = vv;
    }
    j0 = q1;
  }
#pragma unroll 8
  for (int64_t j = j0 + threadIdx.x; j < s1; j += kAdamThreads) upd(g[j], p[j], m[j], v[j]);
}

int64_t blocks_of(int64_t numel, int64_t slice = kSliceElems) { return std::max<int64_t>(1, cdiv(numel, slice)); }

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" size_t aimx_fused_adam_workspace_bytes(const AimxAdamTensor* tensors, int32_t n) {
  if (!tensors || n < 0) return 0;
  int64_t blocks = 0;
  for (int32_t i = 0; i < n; ++i) blocks += blocks_of(tensors[i].numel);
  return sizeof(double) * (size_t)(blocks + 1) + sizeof(float) * 8;
}

extern "C" int aimx_fused_adam(const AimxAdamTensor* tensors, int32_t n, const AimxAdamHyper* h, float* step,
                               const float* lr, float* norm_out, void* workspace, size_t workspace_bytes,
                               aimx_stream_t stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (!tensors || n < 0 || !h || !step || !lr) return AIMX_EARG;
  if (n == 0) return AIMX_OK;
  if (!workspace || workspace_bytes < aimx_fused_adam_workspace_bytes(tensors, n)) return AIMX_EARG;
  for (int32_t i = 0; i < n; ++i) {
    const AimxAdamTensor& x = tensors[i];
    if (x.numel < 0 || (x.numel > 0 && (!x.param || !x.grad || !x.exp_avg || !x.exp_avg_sq)) || x.group < 0 ||
        x.group > 255 || x.step_slot < 0 || x.step_slot >= (1 << 23))
      return AIMX_EARG;
    for (int32_t k = 0; k < i; ++k)  // each counter advanced once per call
      if (tensors[k].step_slot == x.step_slot) return AIMX_EARG;
  }
  // workspace: [8 B, unused (the former arrival counter; keeps the partials' place)] [partials]
  // [scalars]; the partials fit: a slice is never smaller than kSliceElems
  double* partial = (double*)workspace + 1;
  int64_t elems = 0;
  for (int32_t i = 0; i < n; ++i) elems += tensors[i].numel;
  int64_t slice = kSliceElems;
  while (slice < (int64_t(1) << 24) && elems > slice * kTargetSlices) slice *= 2;
  int64_t total_blocks = 0, max_blocks = 0;
  for (int32_t i = 0; i < n; ++i) {
    total_blocks += blocks_of(tensors[i].numel, slice);
    max_blocks += blocks_of(tensors[i].numel);
  }
  float* scal = (float*)(partial + max_blocks);
  // chunk tables (host, by value into the kernel arguments), workgroups of `sl` elements
  auto for_chunks = [&](int64_t sl, auto&& launch) -> int {
    int64_t blk = 0;
    for (int32_t c0 = 0; c0 < n; c0 += kAdamChunk) {
      AdamTable t{};
      t.n = std::min<int32_t>(kAdamChunk, n - c0);
      int32_t b = 0;
      for (int32_t k = 0; k < t.n; ++k) {
        const AimxAdamTensor& x = tensors[c0 + k];
        t.blk0[k] = b;
        t.gs[k] = x.group | (x.step_slot << 8);
        t.numel[k] = x.numel;
        t.param[k] = x.param;
        t.grad[k] = x.grad;
        t.m[k] = x.exp_avg;
        t.v[k] = x.exp_avg_sq;
        b += (int32_t)blocks_of(x.numel, sl);
      }
      t.blk0[t.n] = b;
      const int rc = launch(t, b, blk);
      if (rc) return rc;
      blk += b;
    }
    return AIMX_OK;
  };
  int rc = for_chunks(slice, [&](const AdamTable& t, int32_t nb, int64_t blk) -> int {
    hipLaunchKernelGGL(k_adam_sumsq, dim3((unsigned)nb), dim3(kAdamThreads), 0, s, t, partial, step, blk, slice);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  });
  if (rc) return rc;
  return for_chunks(kSliceElems, [&](const AdamTable& t, int32_t nb, int64_t blk) -> int {
    hipLaunchKernelGGL(k_adam_update, dim3((unsigned)nb), dim3(kAdamThreads), 0, s, t, (const double*)partial,
                       total_blocks, h->max_grad_norm, scal, norm_out, blk == 0 ? 1 : 0, kSliceElems,
                       (const float*)step, lr, h->beta1, h->one_minus_beta1, h->beta2, h->one_minus_beta2, h->eps,
                       h->weight_decay);
    AIMX_CHECK_LAUNCH();
    return AIMX_OK;
  });
}
