// Internal helpers shared by the aimx HIP translation units (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/aimx.h"

#define AIMX_CHECK_HIP(expr)                         \
  do {                                               \
    hipError_t _e = (expr);                          \
    if (_e != hipSuccess) return (int)_e;            \
  } while (0)

#define AIMX_CHECK_LAUNCH() AIMX_CHECK_HIP(hipGetLastError())

namespace aimx {

constexpr int kWave = 64;  // CDNA wavefront

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Path options (version.hip). The product library reads no environment: an option is its default
// unless a test set it through aimx_set_option (include/aimx.h: the alternative-path parity tests),
// and only the tuning build (`make tune`: -DAIMX_TUNING -> lib/libaimx_tune.so, loaded by the tools'
// A/B runs through AIMX_LIB_PATH) also reads the environment variable of the same name.
int64_t opt_i64(const char* name, int64_t dflt);
// A tuning knob (an A/B of a measured variant): read from the environment in the tuning build
// (make tune, -DAIMX_TUNING); the product library always takes the default, so its only
// switchable paths are the opt_i64 options include/aimx.h documents.
#ifdef AIMX_TUNING
inline int64_t tune_i64(const char* name, int64_t dflt) { return opt_i64(name, dflt); }
#else
inline int64_t tune_i64(const char*, int64_t dflt) { return dflt; }
#endif

// Activation kinds (reference: src/utils/activation.py:9-34).
enum Act : int { ACT_NONE = -1, ACT_RELU = 0, ACT_LEAKYRELU = 1, ACT_ELU = 2, ACT_GELU = 3, ACT_SILU = 4 };

__device__ __forceinline__ float act_fwd(int kind, float v) {
  switch (kind) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_LEAKYRELU: return v > 0.f ? v : 0.01f * v;
    case ACT_ELU: return v > 0.f ? v : expm1f(v);
    case ACT_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    // expf and a correctly rounded division: the hardware exp2 / reciprocal form (~4 VALU ops instead
    // of ~22) moved c3's temperature gradient from 0.55x to 3.3x the reference's own fp32 error
    case ACT_SILU: return v / (1.f + expf(-v));
    default: return v;
  }
}

// d act / d v evaluated at the pre-activation v (matches ATen's *_backward formulas).
__device__ __forceinline__ float act_grad(int kind, float v) {
  switch (kind) {
    case ACT_RELU: return v > 0.f ? 1.f : 0.f;
    case ACT_LEAKYRELU: return v > 0.f ? 1.f : 0.01f;
    case ACT_ELU: return v > 0.f ? 1.f : expf(v);
    case ACT_GELU: {
      const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
      const float pdf = expf(-0.5f * v * v) * 0.39894228040143268f;
      return cdf + v * pdf;
    }
    case ACT_SILU: {
      const float s = 1.f / (1.f + expf(-v));
      return s * (1.f + v * (1.f - s));
    }
    default: return 1.f;
  }
}

// Counter-based hash for dropout masks: uniform in [0,1) from (seed, salt, index). The 64-bit seed
// and the salt fold into two 32-bit keys (splitmix64; uniform per call site, so hoisted out of the
// element loops), and each element costs two rounds of a 32-bit integer finaliser over its index
// (lowbias32: 2 multiplies each). The earlier splitmix64 of the index took three 64-bit multiplies
// (12 quarter-rate VALU ops) per element, which made the dropout epilogues VALU-bound (k_mlps c4:
// 8-10 us of an 80 us launch). Rate, lag correlations and per-column rates checked on 2e7 draws.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float hash_uniform(uint64_t seed, uint32_t salt, uint64_t idx) {
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(salt + 1));
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  uint32_t h = mix32((uint32_t)idx ^ (uint32_t)z);
  h = mix32(h ^ (uint32_t)(idx >> 32) ^ (uint32_t)(z >> 32));
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// The n dropout seeds of one forward from the device counter at state (one thread): splitmix64 of
// the counter, in [0, 2^62) like torch.randint(0, 2**62); the counter advances by n + 1 golden
// steps (aimx_dropout_seeds, and the embedding gather's optional seed draw).
__device__ __forceinline__ void draw_dropout_seeds(int64_t* state, int64_t* seeds, int32_t n) {
  const uint64_t s = (uint64_t)state[0];
  for (int32_t i = 0; i < n; ++i) {
    uint64_t z = s + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    seeds[i] = (int64_t)(z >> 2);
  }
  state[0] = (int64_t)(s + 0x9E3779B97F4A7C15ull * (uint64_t)(n + 1));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Raw buffer descriptor over [p, p + bytes) (stride 0, num_records in bytes, dword3 0x00020000 =
// DATA_FORMAT 32): loads past the extent return 0 and stores past it are dropped, so an invalid
// element is an ADDRESS select (offset >= bytes, or kBufDrop) instead of a branch around the access.
// The inputs are made provably wave-uniform with readfirstlane so hipcc builds the descriptor in
// SGPRs and does not waterfall the accesses (guide T8/T20).
//
// The halves MUST pass through uint32_t: __builtin_amdgcn_readfirstlane returns int, and
// `((uint64_t)hi << 32) | readfirstlane(lo)` sign-extends the low half — a base whose bit 31 is set
// becomes 0xFFFF'xxxxxxxx after the descriptor keeps the low 16 bits of the high dword (hipcc:
// s_bfe_i64 + s_or_b64 into the base). That address faults; it is what made the round-4 attention
// pool's two-round row loads fault on one allocation of one test and not on the others.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = (void*)(((uint64_t)hi << 32) | (uint64_t)lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
// A buffer offset past every extent (extents stay below 2^32 - 16, so offset + 12 does not wrap).
constexpr uint32_t kBufDrop = 0xFFFFFFF0u;

// Internal launchers shared across translation units.
// The 8-molecule fused head (head8.hip); head.hip's entry points dispatch to it where it applies.
bool head8_ok(const AimxHead* h);
size_t head8_forward_workspace_floats(const AimxHead* h);
int head8_forward(const AimxHead* h, float* wt, hipStream_t st);
int head8_backward(const AimxHead* h, const AimxHeadGrad* d, hipStream_t st);
// aimx_segment_gather_sum (hop.hip) with skip_tail: chunks in the trailing run of edge-less hop chunks
// are not written (only for consumers that trim them: the stack's GEMMs via AimxGemmArgs.zc_*)
int segment_gather_sum(const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
                       const int32_t* rowptr, const int32_t* col, int64_t rows, float* out, int64_t out_ld,
                       int64_t out_rpc, int64_t out_cs, const float* add0, int64_t add0_ld, const float* add1,
                       int64_t add1_ld, const int64_t* row_seg, int64_t row_seg_stride, hipStream_t stream,
                       int32_t skip_tail);
int launch_gemm(const AimxGemmArgs& a, hipStream_t s);
size_t gemm_workspace_floats(const AimxGemmArgs& a);
int launch_charge_fwd(const float* x, int64_t ldx, int64_t N, int64_t D, const int32_t* gptr, const int32_t* gperm,
                      int64_t G, const float* tc, float* out, int64_t ldo, hipStream_t s);
int launch_charge_bwd(const float* x, int64_t ldx, int64_t N, int64_t D, const int32_t* gptr, const int32_t* gperm,
                      int64_t G, const float* tc, const float* dout, int64_t ldd, float* dx, int64_t lddx,
                      hipStream_t s);

// Fused node-update MLP of one shell layer (mlp.hip): all MLP blocks in one launch each way.
// D > 128 takes the weight-streamed kernels, which read their weights from MFMA-fragment images:
// mlp_pack_floats(s) floats (0: not needed) written by launch_mlp_pack once per call and direction,
// passed as `pack` (nullptr: the weight-resident kernels).
bool mlp_fused_ok(int64_t N, int64_t D, int64_t nm, int32_t precision, int64_t ld);
// the stack's F / UG row strides (AimxShellStack.ld_f / ld_ug; 0 = dense)
inline int64_t stack_ld_f(const AimxShellStack* s) {
  return s->ld_f > 0 ? s->ld_f : s->D * (s->num_hops + 1);
}
inline int64_t stack_ld_ug(const AimxShellStack* s) { return s->ld_ug > 0 ? s->ld_ug : 2 * s->D; }
// row stride of the MLP blocks' R / A activations and of their gradients dV / dA (ld_act; 0 = D)
inline int64_t stack_ld_act(const AimxShellStack* s) { return s->ld_act > 0 ? s->ld_act : s->D; }
size_t mlp_pack_floats(const AimxShellStack* s);
int launch_mlp_pack(const AimxShellStack* s, bool bwd, float* dst, hipStream_t st);
int launch_mlp_fwd(const AimxShellStack* s, int64_t l, const float* x_res, int64_t ldx, float* out, int64_t ldo,
                   const float* pack, hipStream_t st);
int launch_mlp_bwd(const AimxShellStack* s, int64_t l, const float* dy, int64_t lddy, float* const* dV,
                   float* const* dA, float* dug, const float* pack, hipStream_t st);

}  // namespace aimx
