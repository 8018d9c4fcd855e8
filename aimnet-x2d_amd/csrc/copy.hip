// Multi-tensor copy / zero fill in one launch per chunk of items (aimx.h aimx_multi_copy).
//
// The gradient sync of data-parallel training moves every gradient into its bucket's flat RCCL
// buffer and back after the all-reduce. torch.cat + torch._foreach_copy_ did that in three
// launches (8 + 35 + 35 us at c2: the foreach kernel's small chunks over ~70 tensors of 77 to
// 46k floats leave HBM idle). Here the item table rides in the kernel arguments (like
// adam.hip's), each workgroup copies one 4096-float slice of one item, 16 floats per thread in
// flight, with 16-byte accesses when both ends are 16-byte aligned.
#include <algorithm>

#include "aimx_common.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace aimx {
namespace {

constexpr int kChunk = 64;
constexpr int kThreads = 256;
constexpr int64_t kSlice = 4096;

struct CopyTable {
  int32_t n;
  int32_t blk0[kChunk + 1];
  const float* src[kChunk];
  float* dst[kChunk];
  int64_t numel[kChunk];
};
static_assert(sizeof(CopyTable) <= 4000, "kernel argument table must stay under the 4 KiB limit");

__global__ __launch_bounds__(kThreads) void k_multi_copy(const CopyTable t) {
  int i = 0;
  while (i + 1 < t.n && t.blk0[i + 1] <= (int)blockIdx.x) ++i;
  const int64_t s0 = (int64_t)(blockIdx.x - t.blk0[i]) * kSlice;
  const int64_t s1 = min(t.numel[i], s0 + kSlice);
  const float* __restrict__ src = t.src[i];
  float* __restrict__ dst = t.dst[i];
  const bool vec = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0 && ((s1 - s0) & 3) == 0;
  if (vec) {
    const int64_t q0 = s0 / 4, q1 = s1 / 4;
    for (int64_t j = q0 + threadIdx.x; j < q1; j += kThreads) {
      const floatx4 v = src ? reinterpret_cast<const floatx4*>(src)[j] : floatx4{0.f, 0.f, 0.f, 0.f};
      reinterpret_cast<floatx4*>(dst)[j] = v;
    }
  } else {
#pragma unroll 4
    for (int64_t j = s0 + threadIdx.x; j < s1; j += kThreads) dst[j] = src ? src[j] : 0.f;
  }
}

int64_t slices(int64_t n) { return std::max<int64_t>(1, cdiv(n, kSlice)); }

// Dropout seeds of one forward from a device-resident counter (aimx_dropout_seeds).
__global__ void k_dropout_seeds(int64_t* __restrict__ state, int64_t* __restrict__ seeds, int32_t n) {
  if (threadIdx.x != 0) return;
  draw_dropout_seeds(state, seeds, n);
}

// Static padded inputs of one autograph bucket (aimx_pad_batch): real rows copied, slack atoms
// dealt to pad_mols padding molecules of near-equal size (molecule ids G, G+1, ...; the first
// slack % pad_mols take one atom more), slack edges self-pairs spread over the slack atoms — the
// layout of aimx.data.pad_collated, so every real molecule's values are untouched.
__global__ __launch_bounds__(256) void k_pad_batch(const AimxPadBatch p) {
  const int64_t slack = p.Np - p.N;
  const int64_t q = slack / p.pad_mols, r = slack % p.pad_mols;
  const int64_t total = max(max(p.Np, p.Ep), p.G + p.pad_mols);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < p.Np) {
      const bool real = i < p.N;
#pragma unroll
      for (int k = 0; k < 4; ++k) p.out_feat[k * p.Np + i] = real ? p.feat[k][i * p.feat_stride[k]] : 0;
      int64_t m;
      if (real) {
        m = p.batch[i * p.batch_stride];
      } else {
        const int64_t s = i - p.N;
        m = p.G + (s < r * (q + 1) ? s / (q + 1) : r + (s - r * (q + 1)) / q);
      }
      p.out_batch[i] = m;
    }
    if (i < p.Ep) {
      int64_t t, s;
      if (i < p.E) {
        t = p.edges[i * p.edge_s0];
        s = p.edges[i * p.edge_s0 + p.edge_s1];
      } else {
        t = s = p.N + (i - p.E) % slack;
      }
      p.out_edges[2 * i] = t;
      p.out_edges[2 * i + 1] = s;
    }
    if (i < p.G + p.pad_mols) p.out_charges[i] = i < p.G ? p.charges[i * p.charge_stride] : 0.f;
  }
}

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" int aimx_pad_batch(const AimxPadBatch* p, aimx_stream_t stream) {
  if (!p || p->N < 0 || p->E < 0 || p->G < 0 || p->pad_mols < 1 || p->Np <= p->N || p->Ep < p->E) return AIMX_EARG;
  for (int k = 0; k < 4; ++k)
    if ((p->N > 0 && !p->feat[k]) || p->feat_stride[k] < 1) return AIMX_EARG;
  if ((p->N > 0 && !p->batch) || (p->E > 0 && !p->edges) || (p->G > 0 && !p->charges) || !p->out_feat ||
      !p->out_batch || !p->out_edges || !p->out_charges || p->batch_stride < 1 || p->charge_stride < 1)
    return AIMX_EARG;
  const int64_t total = std::max({p->Np, p->Ep, p->G + p->pad_mols});
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(total, 256), 2048);
  hipLaunchKernelGGL(k_pad_batch, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_multi_copy(const AimxCopyItem* items, int32_t n_items, aimx_stream_t stream) {
  if (n_items < 0 || (n_items > 0 && !items)) return AIMX_EARG;
  for (int32_t i = 0; i < n_items; ++i)
    if (items[i].n < 0 || (items[i].n > 0 && !items[i].dst)) return AIMX_EARG;
  for (int32_t c0 = 0; c0 < n_items; c0 += kChunk) {
    CopyTable t{};
    t.n = std::min<int32_t>(kChunk, n_items - c0);
    int32_t b = 0;
    for (int32_t k = 0; k < t.n; ++k) {
      const AimxCopyItem& x = items[c0 + k];
      t.blk0[k] = b;
      t.src[k] = x.src;
      t.dst[k] = x.dst;
      t.numel[k] = x.n;
      b += (int32_t)slices(x.n);
    }
    t.blk0[t.n] = b;
    hipLaunchKernelGGL(k_multi_copy, dim3((unsigned)b), dim3(kThreads), 0, (hipStream_t)stream, t);
    AIMX_CHECK_LAUNCH();
  }
  return AIMX_OK;
}

extern "C" int aimx_dropout_seeds(int64_t* state, int64_t* seeds, int32_t n, aimx_stream_t stream) {
  if (n < 0 || !state || (n > 0 && !seeds)) return AIMX_EARG;
  hipLaunchKernelGGL(k_dropout_seeds, dim3(1), dim3(64), 0, (hipStream_t)stream, state, seeds, n);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
