// Stereochemistry features of the message-passing stack, forward and backward.
//
// Reference: GNN._apply_stereochemistry, src/models/gnn.py:310-326, with
//   _cis_trans_calculation (gnn.py:452-497): ct = x.scatter_add(cis[1] ++ trans[1], -x[cis[0]] ++ x[trans[0]])
//     (rows 0 and 1 of the collated [M, 2] cis / trans tensors, exactly as the reference indexes them);
//   _tetrahedral_feature_calculation_physics_inspired (gnn.py:376-450): for chiral centre m with
//     neighbour rows e_j = x[tet[m][j]] (j = 0..3): u_j = e_j / max(|e_j|, 1e-8),
//     chi_j = s * P(u_{j+1}, u_{j+2}, u_{j+3}) (indices mod 4, P(a,b,c) = a^2(b-c) + b^2(c-a) + c^2(a-b)
//     elementwise), s = tanh(mean_j |e_j| / 3); tet = x.clone().index_add_(0, tet.flat, chi), then rows
//     named by no centre are zeroed.
// The op writes the concatenation [x | ct | tet] ([N, 3D], the input of stereochemical_embedding_2)
// directly. Scatter order is the reference's CPU order (item order), made deterministic by a stable
// CSR of the tetrahedral items (aimx_csr_build) and by the fixed order of the <= 4 cis/trans items:
//   k_stereo_chi  : one wave per centre: norms, scale, the 4 chi rows -> scratch (and the norms / s)
//   k_stereo_rows : one row per wave: [x | x + ct items | keep ? x + sum chi : 0]
// Backward (dC = [dA | dB | dT]):
//   k_stereo_chi_bwd : one wave per centre: G_j = dT[tet[m][j]] -> the 4 neighbour-row gradients
//   k_stereo_rows_bwd: dx[n] = dA + dB + keep*dT + sum over ct items with src n of sign*dB[tgt]
//                      + sum over tetrahedral items at n of their neighbour-row gradient
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

constexpr int kStMaxD = 1024;       // features per row (16 per lane)
constexpr int kStPer = kStMaxD / 64;

struct StereoArgs {
  const float* x;
  int64_t ldx, N, D;
  const int64_t* tet;
  int64_t tet_s0, tet_s1, M;
  const int64_t* ct[2];          // cis, trans [rows, 2] int64 (device); rows 0 / 1 = sources / targets
  int64_t ct_s0[2], ct_s1[2], ct_rows[2];
  const int32_t* t_rowptr;  // CSR of the 4M tetrahedral items keyed by atom row (col = item id)
  const int32_t* t_col;
  float* chi;     // [4M, D] scratch
  float* stats;   // [M, 8]: |e_0..3|, s
  float* out;     // [N, 3D]
  int64_t ldo;
};

__device__ __forceinline__ float P(float a, float b, float c) { return a * a * (b - c) + b * b * (c - a) + c * c * (a - b); }

__device__ __forceinline__ int64_t tet_at(const StereoArgs& a, int64_t m, int j) {
  return a.tet[m * a.tet_s0 + j * a.tet_s1];
}

// The reference's <= 4 cis/trans items in scatter order: cis (sign -1) then trans (sign +1), each
// (source = row 0, target = row 1) at column i = 0, 1. Out-of-range items are skipped (the
// reference would raise an index error).
struct CtItems {
  int64_t src[4], tgt[4];
  float sign[4];
};
__device__ __forceinline__ CtItems ct_items(const StereoArgs& a) {
  CtItems c;
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int slot = 2 * k + i;
      c.sign[slot] = k == 0 ? -1.f : 1.f;
      c.src[slot] = c.tgt[slot] = -1;
      if (a.ct_rows[k] >= 2) {
        const int64_t sv = a.ct[k][i * a.ct_s1[k]], tv = a.ct[k][a.ct_s0[k] + i * a.ct_s1[k]];
        if (sv >= 0 && sv < a.N && tv >= 0 && tv < a.N) {
          c.src[slot] = sv;
          c.tgt[slot] = tv;
        }
      }
    }
  return c;
}

// One wave per centre m.
__global__ __launch_bounds__(256) void k_stereo_chi(const StereoArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int D = (int)a.D;
  float e[4][kStPer];
  float mag[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t r = tet_at(a, m, j);
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < kStPer; ++q) {
      const int d = lane + 64 * q;
      const float v = (d < D && r >= 0 && r < a.N) ? a.x[r * a.ldx + d] : 0.f;
      e[j][q] = v;
      ss += v * v;
    }
    mag[j] = sqrtf(wave_sum(ss));
  }
  const float s = tanhf((((mag[0] + mag[1]) + mag[2]) + mag[3]) * 0.25f / 3.f);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float inv = 1.f / fmaxf(mag[j], 1e-8f);
#pragma unroll
    for (int q = 0; q < kStPer; ++q) e[j][q] *= inv;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float* dst = a.chi + (m * 4 + j) * a.D;
#pragma unroll
    for (int q = 0; q < kStPer; ++q) {
      const int d = lane + 64 * q;
      if (d < D) dst[d] = s * P(e[(j + 1) & 3][q], e[(j + 2) & 3][q], e[(j + 3) & 3][q]);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) a.stats[m * 8 + j] = mag[j];
    a.stats[m * 8 + 4] = s;
  }
}

// One row per wave: the [x | ct | tet] concatenation.
__global__ __launch_bounds__(256) void k_stereo_rows(const StereoArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= a.N) return;
  const int64_t D = a.D;
  const float* xr = a.x + n * a.ldx;
  float* o = a.out + n * a.ldo;
  const bool has_tet = a.M > 0;
  const int32_t tb = has_tet ? a.t_rowptr[n] : 0, te = has_tet ? a.t_rowptr[n + 1] : 0;
  const CtItems ci = ct_items(a);
  for (int64_t d = lane; d < D; d += 64) {
    const float xv = xr[d];
    o[d] = xv;
    float c = xv;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (ci.tgt[i] == n) c += ci.sign[i] * a.x[ci.src[i] * a.ldx + d];
    o[D + d] = c;
    float t = xv;
    if (has_tet) {
      for (int32_t k = tb; k < te; ++k) t += a.chi[(int64_t)a.t_col[k] * D + d];
      if (te == tb) t = 0.f;
    }
    o[2 * D + d] = t;
  }
}

struct StereoGrad {
  const float* dc;  // [N, 3D]
  int64_t lddc;
  float* gx;        // [4M, D] scratch: each tetrahedral item's neighbour-row gradient
  float* dx;        // [N, D]
  int64_t lddx;
};

// One wave per centre: gradients of the 4 chi rows w.r.t. the 4 neighbour rows.
__global__ __launch_bounds__(256) void k_stereo_chi_bwd(const StereoArgs a, const StereoGrad g) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int D = (int)a.D;
  float u[4][kStPer], G[4][kStPer], du[4][kStPer];
  float mag[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) mag[j] = a.stats[m * 8 + j];
  const float s = a.stats[m * 8 + 4];
  float ds = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t r = tet_at(a, m, j);
    const bool ok = r >= 0 && r < a.N;
    const float inv = 1.f / fmaxf(mag[j], 1e-8f);
#pragma unroll
    for (int q = 0; q < kStPer; ++q) {
      const int d = lane + 64 * q;
      const bool in = d < D && ok;
      u[j][q] = in ? a.x[r * a.ldx + d] * inv : 0.f;
      G[j][q] = in ? g.dc[r * g.lddc + 2 * a.D + d] : 0.f;
      du[j][q] = 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float part = 0.f;
#pragma unroll
    for (int q = 0; q < kStPer; ++q) {
      const float A = u[(j + 1) & 3][q], B = u[(j + 2) & 3][q], C = u[(j + 3) & 3][q];
      const float gj = G[j][q];
      part += gj * P(A, B, C);
      const float dcj = s * gj;
      du[(j + 1) & 3][q] += dcj * (2.f * A * (B - C) - B * B + C * C);
      du[(j + 2) & 3][q] += dcj * (A * A + 2.f * B * (C - A) - C * C);
      du[(j + 3) & 3][q] += dcj * (-A * A + B * B + 2.f * C * (A - B));
    }
    ds += wave_sum(part);
  }
  const float dmag = ds * (1.f - s * s) * (1.f / 3.f) * 0.25f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float ud = 0.f;
#pragma unroll
    for (int q = 0; q < kStPer; ++q) ud += u[j][q] * du[j][q];
    ud = wave_sum(ud);
    const float nrm = mag[j];
    float* dst = g.gx + (m * 4 + j) * a.D;
#pragma unroll
    for (int q = 0; q < kStPer; ++q) {
      const int d = lane + 64 * q;
      if (d >= D) continue;
      // u = e / max(|e|, eps): d e = (du - u <u, du>) / |e| above eps, du / eps below;
      // |e|: d e += dmag * e / |e| (0 at e = 0, as torch's norm backward)
      float v = nrm > 1e-8f ? (du[j][q] - u[j][q] * ud) / nrm : du[j][q] * 1e8f;
      if (nrm > 0.f) v += dmag * u[j][q] * (nrm > 1e-8f ? 1.f : 1e-8f / nrm);
      dst[d] = v;
    }
  }
}

// One row per wave.
__global__ __launch_bounds__(256) void k_stereo_rows_bwd(const StereoArgs a, const StereoGrad g) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= a.N) return;
  const int64_t D = a.D;
  const float* dcr = g.dc + n * g.lddc;
  const bool has_tet = a.M > 0;
  const int32_t tb = has_tet ? a.t_rowptr[n] : 0, te = has_tet ? a.t_rowptr[n + 1] : 0;
  const CtItems ci = ct_items(a);
  for (int64_t d = lane; d < D; d += 64) {
    float v = dcr[d] + dcr[D + d];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (ci.src[i] == n) v += ci.sign[i] * g.dc[ci.tgt[i] * g.lddc + D + d];
    if (has_tet) {
      if (te > tb) v += dcr[2 * D + d];
      for (int32_t k = tb; k < te; ++k) v += g.gx[(int64_t)a.t_col[k] * D + d];
    } else {
      v += dcr[2 * D + d];  // no centres: the tetrahedral block is x itself (gnn.py:391-392)
    }
    g.dx[n * g.lddx + d] = v;
  }
}

StereoArgs make_args(const AimxStereo* p) {
  StereoArgs a{};
  a.x = p->x;
  a.ldx = p->ldx;
  a.N = p->N;
  a.D = p->D;
  a.tet = p->tet;
  a.tet_s0 = p->tet_stride0;
  a.tet_s1 = p->tet_stride1;
  a.M = p->M;
  a.ct[0] = p->cis;
  a.ct[1] = p->trans;
  a.ct_rows[0] = p->n_cis;
  a.ct_rows[1] = p->n_trans;
  a.ct_s0[0] = p->cis_stride0;
  a.ct_s1[0] = p->cis_stride1;
  a.ct_s0[1] = p->trans_stride0;
  a.ct_s1[1] = p->trans_stride1;
  a.t_rowptr = p->t_rowptr;
  a.t_col = p->t_col;
  a.chi = p->scratch;
  a.stats = p->stats;
  a.out = p->out;
  a.ldo = p->ldo;
  return a;
}

bool stereo_valid(const AimxStereo* p) {
  if (!p || p->N < 0 || p->D < 1 || p->D > kStMaxD || !p->x || p->ldx < p->D || p->M < 0) return false;
  if ((p->n_cis > 0 && (p->n_cis < 2 || !p->cis)) || (p->n_trans > 0 && (p->n_trans < 2 || !p->trans))) return false;
  if (p->M > 0 && (!p->tet || !p->t_rowptr || !p->t_col || !p->scratch || !p->stats)) return false;
  return true;
}

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" int aimx_stereo_forward(const AimxStereo* p, aimx_stream_t stream) {
  if (!stereo_valid(p) || !p->out || p->ldo < 3 * p->D) return AIMX_EARG;
  if (p->N == 0) return AIMX_OK;
  const StereoArgs a = make_args(p);
  hipStream_t s = (hipStream_t)stream;
  if (p->M > 0) {
    hipLaunchKernelGGL(k_stereo_chi, dim3((unsigned)cdiv(p->M, 4)), dim3(256), 0, s, a);
    AIMX_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_stereo_rows, dim3((unsigned)cdiv(p->N, 4)), dim3(256), 0, s, a);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_stereo_backward(const AimxStereo* p, const float* d_out, int64_t ld_dout, float* dx, int64_t lddx,
                                    float* grad_scratch, aimx_stream_t stream) {
  if (!stereo_valid(p) || !d_out || ld_dout < 3 * p->D || !dx || lddx < p->D) return AIMX_EARG;
  if (p->M > 0 && !grad_scratch) return AIMX_EARG;
  if (p->N == 0) return AIMX_OK;
  const StereoArgs a = make_args(p);
  StereoGrad g{d_out, ld_dout, grad_scratch, dx, lddx};
  hipStream_t s = (hipStream_t)stream;
  if (p->M > 0) {
    hipLaunchKernelGGL(k_stereo_chi_bwd, dim3((unsigned)cdiv(p->M, 4)), dim3(256), 0, s, a, g);
    AIMX_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_stereo_rows_bwd, dim3((unsigned)cdiv(p->N, 4)), dim3(256), 0, s, a, g);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}
