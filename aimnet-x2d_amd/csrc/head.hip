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
#include <cstdlib>

#include "aimx_common.h"

namespace aimx {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kR = 16;          // molecules per workgroup (the MFMA's 16 rows)
constexpr int kBK = 32;         // k slice of one weight-ring slot
constexpr int kP = 8;           // weight slices in flight from global memory (ring slots)
constexpr int kMaxF = 512;      // widest ffn supported (activations [16][2F] stay in LDS: 129 KiB at 512)
constexpr int kS1 = kMaxF + 4;      // LDS row stride of the [16][F] activation buffers (= 4 mod 64:
constexpr int kS2 = 2 * kMaxF + 4;  //  conflict-free ds_read_b128 of A) ... of the [16][2F] ones
constexpr int kMaxBlocks = AIMX_HEAD_MAX_BLOCKS;

// Clustered mode (AimxHead.cluster = S > 1): S workgroups share one 16-molecule tile and split
// every GEMM's 16-column output fragments between them (fragment f -> workgroup f % S), so the
// chain of a tile runs on S CUs. After each GEMM whose output feeds the next one, the cluster
// exchanges that output through HBM (the tensors the kernel writes anyway: y0, hid, z, cat; ds,
// dz, dv, dy0) by the "Valid forms" row-1 hand-off of MI355X_MICROARCH.md: every exchanged value
// is stored sc1, each storing wave drains (vmcnt 0) before the workgroup barrier, one lane adds
// to the cluster's agent-scope arrival counter and polls it with sc1 loads until all S arrived,
// and every load of the exchanged rows is a 16-byte sc1 buffer load. One workgroup per CU (the
// LDS footprint is padded above half a CU's 160 KiB) and grid <= #CUs keep a cluster co-resident;
// every spin is bounded (timeout word sync[0]). Counters count within the launch (target
// S * (phase + 1)) and the last workgroup to finish resets them, so the caller zeroes the sync
// array once, at allocation.
constexpr int kSyncTmo = 0, kSyncDone = 1, kSyncCnt = 4;  // sync word layout (AIMX_HEAD_SYNC_WORDS)
constexpr uint64_t kSpinTicks = 20000000;  // 0.2 s of the 100 MHz wall clock per wait
typedef __attribute__((address_space(1))) int gi32;

struct Cluster {
  int S, rank;    // workgroups per tile and this one's index in its cluster
  int32_t* cnt;   // the cluster's arrival counter (S > 1)
  int32_t* tmo;   // timeout word
  int phase;      // hand-offs done so far in this launch
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const void* p, uint32_t bytes) {
  return buffer_rsrc(p, bytes);  // aimx_common.h (the uint32_t halves matter)
}

// A value another workgroup of the cluster will read: sc1 (write-through) when clustered.
__device__ __forceinline__ void put(const Cluster& cl, float* p, float v) {
  if (cl.S > 1)
    __hip_atomic_store((gi32*)p, __builtin_bit_cast(int, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

// End of a GEMM phase. Unclustered: a workgroup barrier. Clustered: arrive + wait for the
// cluster, then load rows g0.. of `src` (row stride ld floats, ncols columns, rows >= nvalid read
// as 0 by the buffer range check) into the LDS buffer dst (row stride ldl) with sc1 loads.
template <int W>
__device__ __forceinline__ void exchange(Cluster& cl, const float* src, int64_t ld, int nvalid, int ncols,
                                         float* dst, int ldl, int fofs = 0) {
  if (cl.S == 1) {
    __syncthreads();
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add((gi32*)cl.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int target = cl.S * (cl.phase + 1);
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load((gi32*)cl.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > kSpinTicks) {  // give up: flag it, never hang the device
        __hip_atomic_store((gi32*)cl.tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  cl.phase++;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r = head_rsrc(src, (uint32_t)(4 * (int64_t)max(nvalid, 0) * ld));
  // Only the partners' 16-column fragments are loaded: this workgroup's own ones (fragment f + fofs
  // of the producing GEMM belongs to member (f + fofs) % S) are already in dst, written by its
  // epilogue. The j-th foreign fragment of a row is f = (j / (S-1)) * S + j % (S-1), skipping the
  // own residue.
  const int S = cl.S, nf = ncols / 16;  // ncols % 16 == 0
  const int own = ((cl.rank - fofs) % S + S) % S;
  const int nfor = nf - (nf / S + (own < nf % S ? 1 : 0));
  for (int e = threadIdx.x; e < kR * nfor * 4; e += 64 * W) {
    const int row = e / (nfor * 4), q = e - row * (nfor * 4), j = q >> 2;
    const int jj = j % (S - 1), f = (j / (S - 1)) * S + jj + (jj >= own ? 1 : 0);
    const int c = 16 * f + 4 * (q & 3);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(4 * (row * ld + c)), 0, 16);  // sc1
    *reinterpret_cast<floatx4*>(dst + row * ldl + c) = __builtin_bit_cast(floatx4, v);
  }
  __syncthreads();
}

// One GEMM of the chain: B(k, n) = W[n * ldw + k] (k-contiguous weight rows: the forward's
// nn.Linear weights as they are, the backward's transposed copies), N outputs, K % 32 == 0.
struct Job {
  const float* W;
  int64_t ldw;
  int N, K;
};

// A wave's weight stream: kP slices of its fragment's B operand in registers. The chain's weights
// do not depend on its activations, so the stream runs ahead across fragment and GEMM boundaries:
// the last kP loads of a fragment already fetch the first kP slices of the wave's next fragment
// (of this GEMM, or of the next GEMM of the chain, `nxt`), and those loads fly during the epilogue
// and the phase barrier / cluster exchange. Every load is unconditional (clamped addresses; padded
// slots compute with a zero A operand), so the compiler's vmcnt waits keep the ring in flight.
struct Ring {
  floatx4 rg[kP][2];
  bool primed;  // rg holds slots 0..kP-1 of this wave's next fragment
};

// C[16][N] = A[16][K] . B (A in LDS, row stride lda). Output fragment f (columns 16 f + [0, 16))
// belongs to cluster member f % S and, in it, to wave (f / S) % W. The k index inside each
// 16-block is permuted identically for A and B — lane l supplies k = 16 h + 4 (l >> 4) + j at MFMA
// step j of half h — so a lane's B operand of a half is ONE 16-byte global load from weight row
// 16 f + (l & 15) (the two halves of a 32-k slice read whole 128-byte lines: no LDS staging), and
// its A operand one ds_read_b128, read one slot ahead of its MFMAs. The two halves accumulate
// separately (two independent MFMA chains). `pre(row, col)` returns the epilogue's global operands
// of one output (float2: bias, the saved pre-activation, a mask factor ...); it runs BEFORE the k
// loop, so those loads land behind the MFMA work. `epi(row, col, value, pre)` is called once per
// output by the owning thread. No barrier at the end: the caller's exchange() closes the phase.
template <int W, class Pre, class Epi>
__device__ __forceinline__ void chain_gemm(const Cluster& cl, const float* A, int lda, const Job cur, const Job nxt,
                                           Ring& R, Pre pre, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lq = 4 * (lane >> 4);
  auto row = [&](const Job& j, int f) { return j.W + (int64_t)min(16 * f + lr, j.N - 1) * j.ldw + lq; };
  auto ld = [&](const float* r, int sl, floatx4 (&d)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) d[h] = *reinterpret_cast<const floatx4*>(r + sl * kBK + 16 * h);
  };
  const int step = cl.S * W, first = cl.rank + cl.S * wave;
  const int nfrag = (cur.N + 15) / 16, nfrag_n = (nxt.N + 15) / 16;
  const int nsl = cur.K / kBK, NS = (nsl + kP - 1) / kP * kP;  // slots: slices padded to kP
  const int nsl_n = nxt.K / kBK;
  if (first >= nfrag) {  // no fragment here: start the stream of the next GEMM instead
    R.primed = false;
    if (first < nfrag_n) {
      const float* rn = row(nxt, first);
#pragma unroll
      for (int q = 0; q < kP; ++q) ld(rn, min(q, nsl_n - 1), R.rg[q]);
      R.primed = true;
    }
    return;
  }
  for (int f = first; f < nfrag; f += step) {
    // the stream's next fragment: the next of this GEMM, else this wave's first of the next GEMM
    const bool same = f + step < nfrag;
    const bool has_next = same || first < nfrag_n;
    const float* rc = row(cur, f);
    const float* rn = has_next ? row(same ? cur : nxt, same ? f + step : first) : rc;
    const int nsl2 = same ? nsl : (has_next ? nsl_n : nsl);
    if (!R.primed) {
#pragma unroll
      for (int q = 0; q < kP; ++q) ld(rc, min(q, nsl - 1), R.rg[q]);
    }
    const int col = 16 * f + lr;
    float2 pv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) pv[r] = pre((lane >> 4) * 4 + r, min(col, cur.N - 1));
    __builtin_amdgcn_sched_barrier(0);
    floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
    const float* a0 = A + lr * lda + lq;
    floatx4 av[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) av[h] = *reinterpret_cast<const floatx4*>(a0 + 16 * h);
    for (int s0 = 0; s0 < NS; s0 += kP) {
      const bool last = s0 + kP >= NS;  // uniform: this round's reloads feed the next fragment
#pragma unroll
      for (int q = 0; q < kP; ++q) {
        const int sl = s0 + q;
        floatx4 an[2];  // A of the next slot, read before this slot's MFMAs
#pragma unroll
        for (int h = 0; h < 2; ++h) an[h] = *reinterpret_cast<const floatx4*>(a0 + min(sl + 1, nsl - 1) * kBK + 16 * h);
        const bool live = sl < nsl;  // padded slot: zero A, the MFMAs add exact zeros
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const floatx4 a = live ? av[h] : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], R.rg[q][h][j], acc[h], 0, 0, 0);
        }
        ld(last ? rn : rc, last ? min(q, nsl2 - 1) : min(sl + kP, nsl - 1), R.rg[q]);
#pragma unroll
        for (int h = 0; h < 2; ++h) av[h] = an[h];
      }
    }
    R.primed = has_next;
    if (col < cur.N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) epi((lane >> 4) * 4 + r, col, acc[0][r] + acc[1][r], pv[r]);
    }
  }
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

#ifdef AIMX_HEAD_TRACE  // diagnostics build only: phase timestamps of workgroups 0 and grid/2
__device__ long long g_head_trace[2][64];
#define HEAD_STAMP(k)                                                                      \
  do {                                                                                     \
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2) && (k) < 64) \
      g_head_trace[blockIdx.x == 0 ? 0 : 1][(k)] = (long long)wall_clock64();             \
  } while (0)
#else
#define HEAD_STAMP(k) \
  do {                \
  } while (0)
#endif

// LDS: three activation buffers [16][F], [16][F], [16][2F].
// The array is one static size for every variant: 129 KiB (F up to 512), above half of the CU's
// 160 KiB, so a clustered launch gets one workgroup per CU (the hand-off's measured form; see Cluster).
constexpr int kActFloats = 2 * kR * kS1 + kR * kS2;
constexpr int kHeadLdsFloats = std::max(kActFloats, 84 * 1024 / 4);

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

__device__ __forceinline__ Cluster make_cluster(const AimxHead& h) {
  Cluster cl;
  cl.S = max((int)h.cluster, 1);
  cl.rank = (int)blockIdx.x % cl.S;
  cl.cnt = cl.S > 1 ? h.sync + kSyncCnt + blockIdx.x / cl.S : nullptr;
  cl.tmo = cl.S > 1 ? h.sync + kSyncTmo : nullptr;
  cl.phase = 0;
  return cl;
}

// Last workgroup out resets the cluster counters (every wait of the launch is over by then).
__device__ __forceinline__ void cluster_done(const Cluster& cl, const AimxHead& h) {
  if (cl.S == 1) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add((gi32*)(h.sync + kSyncDone), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1) {
      for (int c = 0; c < (int)gridDim.x / cl.S; ++c)
        __hip_atomic_store((gi32*)(h.sync + kSyncCnt + c), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gi32*)(h.sync + kSyncDone), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Clustered: has any wait of this launch (or an earlier one: the word is sticky) given up? Read
// once per tile before the final GEMM; the tile's outputs are then written as NaN, so the per-step
// NaN count of the train loop (aimx.train) catches a lost hand-off on the step it happens instead
// of letting stale rows reach the optimizer. A workgroup that timed out stored the word before its
// next arrival, so a partner released by that arrival reads it too.
__device__ __forceinline__ bool cluster_poisoned(const Cluster& cl, int* s_flag) {
  if (cl.S == 1) return false;
  if (threadIdx.x == 0) *s_flag = __hip_atomic_load((gi32*)cl.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return *s_flag != 0;
}

// Forward. A cluster (or a lone workgroup) walks the 16-molecule tiles tile, tile + #clusters, ...
template <int W>
__global__ __launch_bounds__(64 * W) void k_head_fwd(const AimxHead h) {
  __shared__ __attribute__((aligned(16))) float lds[kHeadLdsFloats];
  __shared__ int s_poison;
  constexpr int NT = 64 * W;
  float* X = lds;                    // current block input y (then z)   [16][kS1]
  float* Hb = X + kR * kS1;          // block hidden h                  [16][kS1]
  float* Cb = Hb + kR * kS1;         // x_pooled, then concat [z | s]   [16][kS2]
  Cluster cl = make_cluster(h);
  const int F = (int)h.F, Hin = (int)h.H_in, T = (int)h.T;
  const int64_t G = h.G;
  const float scale = drop_scale(h.drop_p);
  const bool drop = h.training && h.drop_p > 0.f && h.seed;
  const uint64_t seed = drop ? (uint64_t)*h.seed : 0;
  auto bias = [](const float* b) { return [b](int, int c) { return make_float2(b[c], 0.f); }; };
  const Job jp{h.wp, Hin, F, Hin}, js{h.ws, F, F, F}, jo{h.wo, 2 * F, T, 2 * F};
  auto j1 = [&](int i) { return Job{h.w1[i], F, F, F}; };
  auto j2 = [&](int i) { return Job{h.w2[i], F, F, F}; };
  Ring R;
  R.primed = false;
  int st = 0;
  HEAD_STAMP(st++);
  const int ntiles = (int)cdiv(G, kR), nclusters = (int)gridDim.x / cl.S;
  for (int tile = (int)blockIdx.x / cl.S; tile < ntiles; tile += nclusters) {
    const int64_t g0 = (int64_t)tile * kR;
    const int nvalid = (int)min<int64_t>(kR, G - g0);
    // input rows (x_pooled) -> Cb (as a staging buffer for the first GEMM's A operand)
    for (int e0 = 0; e0 < kR * Hin; e0 += 8 * NT) {  // 8 loads in flight per thread
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * NT + threadIdx.x, r = e / Hin, c = e - r * Hin;
        const bool ok = e < kR * Hin && g0 + r < G;
        v[u] = h.x0[ok ? (g0 + r) * h.ldx0 + c : 0];
        v[u] = ok ? v[u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * NT + threadIdx.x, r = e / Hin, c = e - r * Hin;
        if (e < kR * Hin) Cb[r * kS2 + c] = v[u];
      }
    }
    __syncthreads();
    // y0 = x0 Wp^T + bp
    chain_gemm<W>(cl, Cb, kS2, jp, h.nb ? j1(0) : js, R, bias(h.bp), [&](int r, int c, float v, float2 p) {
      const float y = v + p.x;
      X[r * kS1 + c] = y;
      if (g0 + r < G) put(cl, h.y0 + (g0 + r) * F + c, y);
    });
    HEAD_STAMP(0 + st++);
    exchange<W>(cl, h.y0 + g0 * F, F, nvalid, F, X, kS1);
    HEAD_STAMP(0 + st++);
    for (int i = 0; i < h.nb; ++i) {
      // v = y W1^T + b1 ; h = dropout(act(v))
      float* V = h.v[i];
      float* Hs = h.hid[i];
      uint8_t* M = h.mask[i];
      chain_gemm<W>(cl, X, kS1, j1(i), j2(i), R, bias(h.b1[i]), [&](int r, int c, float acc, float2 p) {
        const float v = acc + p.x;
        float a = act_fwd(h.act, v);
        const int64_t g = g0 + r;
        if (drop) {
          const bool keep =
              hash_uniform(seed, 0x4EADu + (uint32_t)i, (uint64_t)g * (uint64_t)F + (uint64_t)c) >= h.drop_p;
          a = keep ? a * scale : 0.f;
          if (g < G) M[g * F + c] = keep ? 1 : 0;
        }
        Hb[r * kS1 + c] = a;
        if (g < G) {
          V[g * F + c] = v;
          put(cl, Hs + g * F + c, a);
        }
      });
      HEAD_STAMP(0 + st++);
      exchange<W>(cl, Hs + g0 * F, F, nvalid, F, Hb, kS1);
      HEAD_STAMP(0 + st++);
      // z = h W2^T + b2 (+ y)
      float* Z = h.z[i];
      const bool skip = h.skip[i] != 0;
      chain_gemm<W>(cl, Hb, kS1, j2(i), i + 1 < h.nb ? j1(i + 1) : js, R, bias(h.b2[i]), [&](int r, int c, float acc, float2 p) {
        float z = acc + p.x;
        if (skip) z += X[r * kS1 + c];
        X[r * kS1 + c] = z;
        if (g0 + r < G) put(cl, Z + (g0 + r) * F + c, z);
      });
      HEAD_STAMP(0 + st++);
      exchange<W>(cl, Z + g0 * F, F, nvalid, F, X, kS1);
      HEAD_STAMP(0 + st++);
    }
    // s = z Ws^T + bs ; concat [z | s] (the z half of cat is written by cluster member 0 only)
    for (int e = threadIdx.x; e < kR * F; e += NT) {
      const int r = e / F, c = e - r * F;
      Cb[r * kS2 + c] = X[r * kS1 + c];
      if (cl.rank == 0 && g0 + r < G) h.cat[(g0 + r) * 2 * F + c] = X[r * kS1 + c];
    }
    // (the copy above is ordered before the output GEMM by the exchange below; X is only read)
    chain_gemm<W>(cl, X, kS1, js, jo, R, bias(h.bs), [&](int r, int c, float acc, float2 p) {
      const float s = acc + p.x;
      Cb[r * kS2 + F + c] = s;
      if (g0 + r < G) put(cl, h.cat + (g0 + r) * 2 * F + F + c, s);
    });
    HEAD_STAMP(0 + st++);
    exchange<W>(cl, h.cat + g0 * 2 * F + F, 2 * F, nvalid, F, Cb + F, kS2);
    HEAD_STAMP(0 + st++);
    // out = [z | s] Wo^T + bo
    const bool bad = cluster_poisoned(cl, &s_poison);
    chain_gemm<W>(cl, Cb, kS2, jo, jp, R, bias(h.bo), [&](int r, int c, float acc, float2 p) {
      if (g0 + r < G) h.out[(g0 + r) * h.ldo + c] = bad ? __builtin_nanf("") : acc + p.x;
    });
    HEAD_STAMP(0 + st++);
    __syncthreads();  // the next tile overwrites Cb
  }
  HEAD_STAMP(st++);
  cluster_done(cl, h);
  (void)st;
}

// Input-gradient chain. LDS: the staged weight slices + dZ, dS/dV, dO activation buffers.
template <int W>
__global__ __launch_bounds__(64 * W) void k_head_bwd(const AimxHead h, const AimxHeadGrad d) {
  __shared__ __attribute__((aligned(16))) float lds[kHeadLdsFloats];
  __shared__ int s_poison;
  constexpr int NT = 64 * W;
  float* DZ = lds;                    // gradient w.r.t. the current block output  [16][kS1]
  float* DV = DZ + kR * kS1;          // ds, then dv of each block                [16][kS1]
  float* DO = DV + kR * kS1;          // d_out rows                               [16][kS2]
  Cluster cl = make_cluster(h);
  const int F = (int)h.F, Hin = (int)h.H_in, T = (int)h.T;
  const int64_t G = h.G;
  const int Tp = (T + 31) / 32 * 32;
  const HeadWs L = head_ws(F, Hin, T, h.nb);
  const float* wt = (const float*)d.workspace;
  const float scale = drop_scale(h.drop_p);
  const bool drop = h.training && h.drop_p > 0.f && h.seed;
  auto none = [](int, int) { return make_float2(0.f, 0.f); };
  const int last = h.nb - 1;
  const Job jo{wt + L.wo, Tp, 2 * F, Tp}, js{wt + L.ws, F, F, F}, jp{wt + L.wp, F, Hin, F};
  auto j2 = [&](int i) { return Job{wt + L.w2 + 2 * (int64_t)i * F * F, F, F, F}; };
  auto j1 = [&](int i) { return Job{wt + L.w1 + 2 * (int64_t)i * F * F, F, F, F}; };
  Ring R;
  R.primed = false;
  int st = 0;
  HEAD_STAMP(32 + st++);
  const int ntiles = (int)cdiv(G, kR), nclusters = (int)gridDim.x / cl.S;
  for (int tile = (int)blockIdx.x / cl.S; tile < ntiles; tile += nclusters) {
    const int64_t g0 = (int64_t)tile * kR;
    const int nvalid = (int)min<int64_t>(kR, G - g0);
    for (int e = threadIdx.x; e < kR * Tp; e += NT) {
      const int r = e / Tp, c = e - r * Tp;
      DO[r * kS2 + c] = (g0 + r < G && c < T) ? d.d_out[(g0 + r) * d.ld_dout + c] : 0.f;
    }
    __syncthreads();
    // d[z | s] = d_out Wo: dz (direct, own columns only) -> DZ, ds -> DV and HBM
    chain_gemm<W>(cl, DO, kS2, jo, js, R, none, [&](int r, int c, float v, float2) {
      if (c < F) {
        DZ[r * kS1 + c] = v;
      } else {
        DV[r * kS1 + c - F] = v;
        if (g0 + r < G) put(cl, d.ds + (g0 + r) * F + c - F, v);
      }
    });
    HEAD_STAMP(32 + st++);
    exchange<W>(cl, d.ds + g0 * F, F, nvalid, F, DV, kS1, F / 16);  // ds = fragments F/16.. of [dz | ds]
    HEAD_STAMP(32 + st++);
    // dz += ds Ws (fragment f of this GEMM has the owner of fragment f of the one above: the
    // direct dz columns it adds are in this workgroup's LDS)
    chain_gemm<W>(cl, DV, kS1, js, j2(last), R, none, [&](int r, int c, float v, float2) {
      const float z = DZ[r * kS1 + c] + v;
      DZ[r * kS1 + c] = z;
      if (g0 + r < G) put(cl, d.dz[last] + (g0 + r) * F + c, z);
    });
    HEAD_STAMP(32 + st++);
    exchange<W>(cl, d.dz[last] + g0 * F, F, nvalid, F, DZ, kS1);
    HEAD_STAMP(32 + st++);
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
      chain_gemm<W>(cl, DZ, kS1, j2(i), j1(i), R, dpre,
                    [&](int r, int c, float acc, float2 p) {
                      const int64_t g = g0 + r;
                      float dv = 0.f;
                      if (g < G) {
                        dv = acc * p.y * p.x;
                        put(cl, d.dv[i] + g * F + c, dv);
                      }
                      DV[r * kS1 + c] = dv;
                    });
                    HEAD_STAMP(32 + st++);
      exchange<W>(cl, d.dv[i] + g0 * F, F, nvalid, F, DV, kS1);
      HEAD_STAMP(32 + st++);
      // dy = dv W1 (+ dz for a skip block): the gradient w.r.t. this block's input
      const bool skip = h.skip[i] != 0;
      float* dst = i > 0 ? d.dz[i - 1] : d.dy0;
      chain_gemm<W>(cl, DV, kS1, j1(i), i > 0 ? j2(i - 1) : jp, R, none,
                    [&](int r, int c, float acc, float2) {
                      float y = acc;
                      if (skip) y += DZ[r * kS1 + c];
                      DZ[r * kS1 + c] = y;
                      if (g0 + r < G) put(cl, dst + (g0 + r) * F + c, y);
                    });
                    HEAD_STAMP(32 + st++);
      exchange<W>(cl, dst + g0 * F, F, nvalid, F, DZ, kS1);
      HEAD_STAMP(32 + st++);
    }
    // d x_pooled = dy0 Wp
    const bool bad = cluster_poisoned(cl, &s_poison);
    chain_gemm<W>(cl, DZ, kS1, jp, jo, R, none, [&](int r, int c, float acc, float2) {
      if (g0 + r < G) d.d_x0[(g0 + r) * d.ld_dx0 + c] = bad ? __builtin_nanf("") : acc;
    });
    HEAD_STAMP(32 + st++);
    __syncthreads();  // the next tile overwrites DO
  }
  HEAD_STAMP(32 + st++);
  cluster_done(cl, h);
  (void)st;
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
  if (h->cluster < 0 || h->cluster > 8 || (h->cluster & (h->cluster - 1)) || (h->cluster > 1 && !h->sync))
    return false;
  if (h->cluster > 1) {  // exchanged tensors: 16-byte rows for the sc1 b128 loads
    if (!al(h->y0) || !al(h->cat)) return false;
    for (int i = 0; i < h->nb; ++i)
      if (!al(h->hid[i]) || !al(h->z[i])) return false;
  }
  for (int i = 0; i < h->nb; ++i)
    if (!al(h->w1[i]) || !al(h->w2[i])) return false;
  return true;
}

struct HeadLaunch {
  unsigned grid;
  int waves;
};

// Clustered: S workgroups of 16 / S waves (at least 4) per tile, #clusters <= #CUs / S (one
// workgroup per CU, see Cluster) and <= the sync array's counters; the clusters walk the tiles.
HeadLaunch head_launch(const AimxHead* h) {
  const int S = std::max((int)h->cluster, 1);
  const int64_t ntiles = cdiv(h->G, kR);
  // waves per workgroup: 8 up to S = 2, then 4 (measured at c2: 1w8 222 us, 2w8 199 us, 2w4 237 us,
  // 4w4 218 us forward+backward; 16 waves need more than the 128 VGPRs a 1024-thread workgroup
  // allows and spill)
  int waves = S <= 2 ? 8 : 4;
  if (const int64_t f = tune_i64("AIMX_HEAD_WAVES", 0)) waves = f == 16 ? 16 : f == 4 ? 4 : 8;  // tuning build
  if (S == 1) return HeadLaunch{(unsigned)ntiles, waves};
  static int cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  const int64_t nc = std::min<int64_t>({ntiles, cus[dev] / S, AIMX_HEAD_SYNC_WORDS - kSyncCnt});
  return HeadLaunch{(unsigned)(std::max<int64_t>(nc, 1) * S), waves};
}

}  // namespace
}  // namespace aimx

extern "C" size_t aimx_head_forward_workspace_bytes(const AimxHead* h) {
  if (!head_valid(h) || !head8_ok(h)) return 0;
  return sizeof(float) * head8_forward_workspace_floats(h);
}

extern "C" int aimx_head_forward(const AimxHead* h, aimx_stream_t stream) {
  if (!head_valid(h)) return AIMX_EARG;
  if (h->G == 0) return AIMX_OK;
  if (head8_ok(h) && h->fwd_ws && h->fwd_ws_bytes >= aimx_head_forward_workspace_bytes(h) &&
      ((uintptr_t)h->fwd_ws & 15) == 0)
    return head8_forward(h, h->fwd_ws, (hipStream_t)stream);
  const HeadLaunch L = head_launch(h);
  switch (L.waves) {
    case 4: hipLaunchKernelGGL(k_head_fwd<4>, dim3(L.grid), dim3(256), 0, (hipStream_t)stream, *h); break;
    case 8: hipLaunchKernelGGL(k_head_fwd<8>, dim3(L.grid), dim3(512), 0, (hipStream_t)stream, *h); break;
    default: hipLaunchKernelGGL(k_head_fwd<16>, dim3(L.grid), dim3(1024), 0, (hipStream_t)stream, *h);
  }
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

#ifdef AIMX_HEAD_TRACE
extern "C" int aimx_head_trace_read(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_head_trace), sizeof(long long) * 128) == hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t aimx_head_backward_workspace_bytes(const AimxHead* h) {
  if (!head_valid(h)) return 0;
  // the 16-molecule kernels' transposes, or the 8-molecule kernels' packed images (head8.hip)
  const size_t t = (size_t)head_ws(h->F, h->H_in, h->T, h->nb).total;
  return sizeof(float) * (head8_ok(h) ? std::max(t, head8_forward_workspace_floats(h)) : t);
}

extern "C" int aimx_head_backward(const AimxHead* h, const AimxHeadGrad* d, aimx_stream_t stream) {
  if (!head_valid(h) || !d || !d->d_out || d->ld_dout < h->T || !d->d_x0 || d->ld_dx0 < h->H_in || !d->ds ||
      !d->dy0 || !d->workspace || d->workspace_bytes < aimx_head_backward_workspace_bytes(h) ||
      ((uintptr_t)d->workspace & 15))
    return AIMX_EARG;
  for (int i = 0; i < h->nb; ++i)
    if (!d->dz[i] || !d->dv[i]) return AIMX_EARG;
  if (h->G == 0) return AIMX_OK;
  if (head8_ok(h)) return head8_backward(h, d, (hipStream_t)stream);  // packs W into the workspace
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
  const HeadLaunch HL = head_launch(h);
  switch (HL.waves) {
    case 4: hipLaunchKernelGGL(k_head_bwd<4>, dim3(HL.grid), dim3(256), 0, (hipStream_t)stream, *h, *d); break;
    case 8: hipLaunchKernelGGL(k_head_bwd<8>, dim3(HL.grid), dim3(512), 0, (hipStream_t)stream, *h, *d); break;
    default: hipLaunchKernelGGL(k_head_bwd<16>, dim3(HL.grid), dim3(1024), 0, (hipStream_t)stream, *h, *d);
  }
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
