// Atom-feature embeddings (reference src/models/gnn.py:262-274: four nn.Embedding lookups + cat)
// and elementwise activation backward.
//
// Forward: E[j, t*dim + c] = table_t[index_t[j], c] — one coalesced pass writing the concatenated
// [N, T*dim] matrix the embedding projection GEMM consumes.
// Backward (deterministic, no float atomics): the tables are tiny (119/9/7/7 rows x 64), so each
// workgroup accumulates a chunk of atoms into a private copy of ALL tables in LDS — thread (t, c)
// owns column c of table t, so it is the only writer of those LDS words and adds its chunk's
// rows in atom order — then writes the partial tables; a second kernel sums the partials in a
// fixed order (4 interleaved in-order wave sums, then wave order), so results are identical run to
// run. PyTorch's embedding backward instead sorts the indices (radix sort + segment offsets,
// several launches per table).
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

constexpr int kChunk = 64;   // min atoms per workgroup in the backward (>= 2 workgroups per CU at c2)
constexpr int64_t kMaxChunks = 2048;  // bounds the partial-table workspace for very large batches
inline int64_t chunk_of(int64_t N) { return std::max<int64_t>(kChunk, cdiv(std::max<int64_t>(N, 1), kMaxChunks)); }
constexpr int kUnroll = 8;   // atoms whose index + gradient loads are in flight together
constexpr int kReduceCols = 64, kReduceWaves = 4;

__global__ void k_embed_gather(AimxEmbeddingTables t, int64_t N, float* __restrict__ out, int64_t ldo) {
  if (t.n_seeds > 0 && blockIdx.x == 0 && threadIdx.x == 0) draw_dropout_seeds(t.seed_state, t.seeds, t.n_seeds);
  const int64_t width = (int64_t)t.n_tables * t.dim;
  const int64_t total = N * width;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i / width, k = i - j * width;
    const int tb = (int)(k / t.dim);
    const int64_t c = k - (int64_t)tb * t.dim;
    const int64_t r = t.index[tb][j];
    out[j * ldo + k] = (r >= 0 && r < t.rows[tb]) ? t.table[tb][r * t.dim + c] : 0.f;
  }
}

// 16-byte form of k_embed_gather (dim % 4 == 0, ldo % 4 == 0, 16-byte aligned out and tables,
// N * width < 2^31): one float4 of one table row per thread, 32-bit index math (the int64
// divisions of the generic form cost more than its loads).
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void k_embed_gather4(AimxEmbeddingTables t, int32_t N, float* __restrict__ out, int32_t ldo) {
  if (t.n_seeds > 0 && blockIdx.x == 0 && threadIdx.x == 0) draw_dropout_seeds(t.seed_state, t.seeds, t.n_seeds);
  const int32_t q = t.dim >> 2, wq = t.n_tables * q, total = N * wq;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int32_t j = i / wq, k = i - j * wq, tb = k / q, c = 4 * (k - tb * q);
    const int64_t r = t.index[tb][j];
    const bool ok = r >= 0 && r < t.rows[tb];
    const floatx4 v = *reinterpret_cast<const floatx4*>(t.table[tb] + (ok ? r : 0) * t.dim + c);
    *reinterpret_cast<floatx4*>(out + (int64_t)j * ldo + tb * t.dim + c) = ok ? v : floatx4{0.f, 0.f, 0.f, 0.f};
  }
}

// 16-byte form of k_act_bwd (N, ldy, ldp, ldo % 4 == 0, aligned pointers, M * N < 2^31).
__global__ void k_act_bwd4(int kind, const float* __restrict__ dy, int32_t ldy, const float* __restrict__ pre,
                           int32_t ldp, int32_t M, int32_t N, float* __restrict__ out, int32_t ldo) {
  const int32_t q = N >> 2, total = M * q;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int32_t m = i / q, n = 4 * (i - m * q);
    const floatx4 d = *reinterpret_cast<const floatx4*>(dy + (int64_t)m * ldy + n);
    const floatx4 p = *reinterpret_cast<const floatx4*>(pre + (int64_t)m * ldp + n);
    floatx4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = d[e] * act_grad(kind, p[e]);
    *reinterpret_cast<floatx4*>(out + (int64_t)m * ldo + n) = o;
  }
}

// Two-source form: columns [0, n0) of dy come from dy0 (ld ldy0), columns [n0, N) from dy1 (ld
// ldy1, column n -> dy1[n - n0]); pre / out rows hold N % 4 == 0 floats at 16-byte-aligned starts.
// One float4 of pre / out per thread; dy is read as a float4 where the source's 4 columns are
// 16-byte aligned and inside one part, else element by element (the split of gnn.py:227-231 at
// hidden 512 / 1024 puts both parts at odd column counts).
__global__ void k_act_bwd2(int kind, const float* __restrict__ dy0, int32_t ldy0, int32_t n0,
                           const float* __restrict__ dy1, int32_t ldy1, const float* __restrict__ pre, int32_t ldp,
                           int32_t M, int32_t N, float* __restrict__ out, int32_t ldo) {
  const int32_t q = N >> 2, total = M * q;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int32_t m = i / q, n = 4 * (i - m * q);
    const floatx4 p = *reinterpret_cast<const floatx4*>(pre + (int64_t)m * ldp + n);
    floatx4 d;
    const float* s0 = dy0 + (int64_t)m * ldy0 + n;
    const float* s1 = dy1 + (int64_t)m * ldy1 + (n - n0);
    if (n + 4 <= n0 && ((uintptr_t)s0 & 15) == 0) {
      d = *reinterpret_cast<const floatx4*>(s0);
    } else if (n >= n0 && ((uintptr_t)s1 & 15) == 0) {
      d = *reinterpret_cast<const floatx4*>(s1);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = (n + e < n0) ? s0[e] : s1[e];
    }
    floatx4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = d[e] * act_grad(kind, p[e]);
    *reinterpret_cast<floatx4*>(out + (int64_t)m * ldo + n) = o;
  }
}

// blockDim.x == n_tables * dim (<= 1024); dynamic LDS = total_rows * dim floats.
__global__ void k_embed_bwd_partial(AimxEmbeddingTables t, int64_t N, int64_t chunk, const float* __restrict__ dE,
                                    int64_t ldd, float* __restrict__ partial, int64_t total_rows) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tb = threadIdx.x / (int)t.dim;
  const int c = threadIdx.x - tb * (int)t.dim;
  int64_t row0 = 0;
  for (int i = 0; i < tb; ++i) row0 += t.rows[i];
  for (int64_t i = threadIdx.x; i < total_rows * t.dim; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int64_t j0 = (int64_t)blockIdx.x * chunk, j1 = min(N, j0 + chunk);
  const int64_t rows_tb = t.rows[tb];
  const int64_t* __restrict__ idx = t.index[tb];
  const float* __restrict__ g = dE + (int64_t)tb * t.dim + c;
  // Loads are unconditional (clamped atom, clamped row) so 2*kUnroll of them are in flight; the
  // LDS adds then run in atom order with a select, which keeps the sum sequential per column.
  for (int64_t j = j0; j < j1; j += kUnroll) {
    int64_t r[kUnroll];
    float v[kUnroll];
#pragma unroll
    for (int q = 0; q < kUnroll; ++q) {
      const int64_t jj = min(j + q, j1 - 1);
      r[q] = idx[jj];
      v[q] = g[jj * ldd];
    }
#pragma unroll
    for (int q = 0; q < kUnroll; ++q) {
      const bool ok = (j + q < j1) && r[q] >= 0 && r[q] < rows_tb;
      const int64_t rr = ok ? r[q] : 0;
      float* cell = &lds[(row0 + rr) * t.dim + c];
      const float cur = *cell;
      *cell = ok ? cur + v[q] : cur;
    }
  }
  __syncthreads();
  float* out = partial + (int64_t)blockIdx.x * total_rows * t.dim;
  for (int64_t i = threadIdx.x; i < total_rows * t.dim; i += blockDim.x) out[i] = lds[i];
}

// Column sums over the per-chunk partial tables: a workgroup owns kReduceCols consecutive table
// words; wave w sums chunks w, w+4, ... in order, then the 4 wave sums are added in wave order
// (a fixed order: deterministic run to run).
__global__ __launch_bounds__(kReduceCols * kReduceWaves) void k_embed_bwd_reduce(AimxEmbeddingTables t,
                                                                               const float* __restrict__ partial,
                                                                               int64_t nblk, int64_t total_rows) {
  __shared__ float part[kReduceWaves][kReduceCols];
  const int64_t total = total_rows * t.dim;
  const int lane = threadIdx.x % kReduceCols, w = threadIdx.x / kReduceCols;
  const int64_t i = (int64_t)blockIdx.x * kReduceCols + lane;
  const int64_t ic = min(i, total - 1);
  float s = 0.f;
  int64_t b = w;
  for (; b + 3 * kReduceWaves < nblk; b += 4 * kReduceWaves) {
    const float a0 = partial[b * total + ic], a1 = partial[(b + kReduceWaves) * total + ic];
    const float a2 = partial[(b + 2 * kReduceWaves) * total + ic], a3 = partial[(b + 3 * kReduceWaves) * total + ic];
    s += a0;
    s += a1;
    s += a2;
    s += a3;
  }
  for (; b < nblk; b += kReduceWaves) s += partial[b * total + ic];
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && i < total) {
    float acc = part[0][lane];
    for (int q = 1; q < kReduceWaves; ++q) acc += part[q][lane];
    int64_t r = i / t.dim;
    const int64_t c = i - r * t.dim;
    int tb = 0;
    while (r >= t.rows[tb]) r -= t.rows[tb++];
    t.grad[tb][r * t.dim + c] = acc;
  }
}

__global__ void k_zero_f32(float* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0.f;
}

__global__ void k_act_bwd(int kind, const float* __restrict__ dy, int64_t ldy, const float* __restrict__ pre,
                          int64_t ldp, int64_t M, int64_t N, float* __restrict__ out, int64_t ldo) {
  const int64_t total = M * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N, n = i - m * N;
    out[m * ldo + n] = dy[m * ldy + n] * act_grad(kind, pre[m * ldp + n]);
  }
}

int64_t total_rows_of(const AimxEmbeddingTables* t) {
  int64_t s = 0;
  for (int i = 0; i < t->n_tables; ++i) s += t->rows[i];
  return s;
}

bool tables_ok(const AimxEmbeddingTables* t) {
  if (!t || t->n_tables < 1 || t->n_tables > AIMX_MAX_TABLES || t->dim < 1) return false;
  if ((int64_t)t->n_tables * t->dim > 1024) return false;
  for (int i = 0; i < t->n_tables; ++i)
    if (t->rows[i] < 1 || !t->index[i]) return false;
  return total_rows_of(t) * t->dim * (int64_t)sizeof(float) <= 160 * 1024;
}

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" int aimx_embedding_gather(const AimxEmbeddingTables* t, int64_t N, float* out, int64_t ldo,
                                     aimx_stream_t s) {
  if (!tables_ok(t) || N < 0 || !out || (t->n_seeds > 0 && (!t->seed_state || !t->seeds)) || t->n_seeds < 0)
    return AIMX_EARG;
  if (N == 0 && t->n_seeds == 0) return AIMX_OK;
  const int64_t total = N * t->n_tables * t->dim;
  bool v4 = t->dim % 4 == 0 && ldo % 4 == 0 && ((uintptr_t)out & 15) == 0 && total < (int64_t)INT32_MAX &&
            N * ldo < (int64_t)INT32_MAX;
  for (int i = 0; i < t->n_tables; ++i) v4 = v4 && ((uintptr_t)t->table[i] & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(k_embed_gather4, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(total / 4, 256), 8192))), dim3(256), 0,
                       (hipStream_t)s, *t, (int32_t)N, out, (int32_t)ldo);
  else
    hipLaunchKernelGGL(k_embed_gather, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(total, 256), 8192))), dim3(256), 0,
                       (hipStream_t)s, *t, N, out, ldo);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" size_t aimx_embedding_backward_workspace_bytes(const AimxEmbeddingTables* t, int64_t N) {
  if (!tables_ok(t)) return 0;
  return sizeof(float) * (size_t)(cdiv(std::max<int64_t>(N, 1), chunk_of(N)) * total_rows_of(t) * t->dim);
}

extern "C" int aimx_embedding_backward(const AimxEmbeddingTables* t, int64_t N, const float* dE, int64_t ldd,
                                       void* ws, size_t ws_bytes, aimx_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (!tables_ok(t) || N < 0) return AIMX_EARG;
  for (int i = 0; i < t->n_tables; ++i)
    if (!t->grad[i]) return AIMX_EARG;
  const int64_t tr = total_rows_of(t);
  if (N == 0) {  // no atoms: zero gradients (by kernel; no runtime memset nodes in captured graphs)
    for (int i = 0; i < t->n_tables; ++i) {
      const int64_t cnt = t->rows[i] * t->dim;
      hipLaunchKernelGGL(k_zero_f32, dim3((unsigned)std::min<int64_t>(cdiv(cnt, 256), 1024)), dim3(256), 0, s,
                         t->grad[i], cnt);
      AIMX_CHECK_LAUNCH();
    }
    return AIMX_OK;
  }
  if (ws_bytes < aimx_embedding_backward_workspace_bytes(t, N) || !ws) return AIMX_EARG;
  const int64_t chunk = chunk_of(N);
  const int64_t nblk = cdiv(N, chunk);
  const size_t lds = sizeof(float) * (size_t)(tr * t->dim);
  hipLaunchKernelGGL(k_embed_bwd_partial, dim3((unsigned)nblk), dim3((unsigned)(t->n_tables * t->dim)), lds, s, *t, N,
                     chunk, dE, ldd, (float*)ws, tr);
  AIMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_embed_bwd_reduce, dim3((unsigned)cdiv(tr * t->dim, kReduceCols)),
                     dim3(kReduceCols * kReduceWaves), 0, s, *t,
                     (const float*)ws, nblk, tr);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_act_backward(int32_t kind, const float* dy, int64_t ldy, const float* pre, int64_t ldp, int64_t M,
                                 int64_t N, float* out, int64_t ldo, aimx_stream_t s) {
  if (M < 0 || N < 0) return AIMX_EARG;
  if (M == 0 || N == 0) return AIMX_OK;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (N % 4 == 0 && ldy % 4 == 0 && ldp % 4 == 0 && ldo % 4 == 0 && al(dy) && al(pre) && al(out) &&
      M * std::max({ldy, ldp, ldo}) < (int64_t)INT32_MAX)
    hipLaunchKernelGGL(k_act_bwd4, dim3((unsigned)std::min<int64_t>(cdiv(M * N / 4, 256), 8192)), dim3(256), 0,
                       (hipStream_t)s, (int)kind, dy, (int32_t)ldy, pre, (int32_t)ldp, (int32_t)M, (int32_t)N, out,
                       (int32_t)ldo);
  else
    hipLaunchKernelGGL(k_act_bwd, dim3((unsigned)std::min<int64_t>(cdiv(M * N, 256), 8192)), dim3(256), 0,
                       (hipStream_t)s, (int)kind, dy, ldy, pre, ldp, M, N, out, ldo);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_act_backward2(int32_t kind, const float* dy0, int64_t ldy0, int64_t n0, const float* dy1,
                                  int64_t ldy1, const float* pre, int64_t ldp, int64_t M, int64_t N, float* out,
                                  int64_t ldo, aimx_stream_t s) {
  if (M < 0 || N < 0 || n0 < 0 || n0 > N) return AIMX_EARG;
  if (M == 0 || N == 0) return AIMX_OK;
  if ((n0 > 0 && !dy0) || (n0 < N && !dy1) || !pre || !out) return AIMX_EARG;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (N % 4 || ldp % 4 || ldo % 4 || !al(pre) || !al(out) || M * std::max({ldy0, ldy1, ldp, ldo}) >= (int64_t)INT32_MAX ||
      ((uintptr_t)dy0 & 3) || ((uintptr_t)dy1 & 3))
    return AIMX_EARG;
  hipLaunchKernelGGL(k_act_bwd2, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(M * N / 4, 256), 8192))),
                     dim3(256), 0, (hipStream_t)s, (int)kind, dy0, (int32_t)ldy0, (int32_t)n0, dy1, (int32_t)ldy1, pre,
                     (int32_t)ldp, (int32_t)M, (int32_t)N, out, (int32_t)ldo);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
