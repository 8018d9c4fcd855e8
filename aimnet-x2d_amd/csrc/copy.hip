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
  const uint64_t s = (uint64_t)state[0];
  for (int32_t i = 0; i < n; ++i) {
    uint64_t z = s + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    seeds[i] = (int64_t)(z >> 2);  // [0, 2^62), the range torch.randint(0, 2**62) drew
  }
  state[0] = (int64_t)(s + 0x9E3779B97F4A7C15ull * (uint64_t)(n + 1));
}

}  // namespace
}  // namespace aimx

using namespace aimx;

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
