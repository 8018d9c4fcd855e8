// Fused L1 losses of the train step (one launch forward, one launch backward).
//
// Reference: trainer._setup_loss_function, src/training/trainer.py:24-35 — nn.L1Loss() for a
// single task (mean |y_pred - y_true| over all elements) and WeightedL1Loss for multitask,
// src/models/losses.py:14-48 (sum over tasks of w_t |y_pred - y_true|, mean over samples). Both are
//   loss = (1 / div) * sum_{i,t} w_t |p_it - y_it|   (w = 1, div = rows*cols | w, div = rows)
// and d p_it = sign(p_it - y_it) * w_t * dloss / div (sign(0) = 0, as ATen's l1_loss backward).
// The forward is one workgroup (the loss is per molecule: rows*cols is a few thousand) with a
// fixed reduction order, so it is deterministic.
#include <algorithm>

#include "aimx_common.h"

namespace aimx {
namespace {

// acc != NULL: also the train step's device-side bookkeeping (aimx_l1_loss_forward_accum):
// acc->loss_sum += loss * acc_scale (two roundings, as torch's mul then add_), acc->nan_count += any
// element of pred[:rows] is NaN, acc->steps += 1.
__global__ __launch_bounds__(256) void k_l1_fwd(const float* __restrict__ p, int64_t ldp, const float* __restrict__ y,
                                                int64_t ldy, int64_t rows, int64_t cols,
                                                const float* __restrict__ w, float inv_div, float* __restrict__ loss,
                                                AimxLossAccum acc) {
  __shared__ float part[4], nanp[4];
  float s = 0.f, nn = 0.f;
  const int64_t n = rows * cols;
  for (int64_t e = threadIdx.x; e < n; e += 256) {
    const int64_t i = e / cols, t = e - i * cols;
    const float pv = p[i * ldp + t];
    const float d = fabsf(pv - y[i * ldy + t]);
    s += w ? d * w[t] : d;
    nn += (pv != pv) ? 1.f : 0.f;
  }
  s = wave_sum(s);
  nn = wave_sum(nn);
  if ((threadIdx.x & 63) == 0) {
    part[threadIdx.x >> 6] = s;
    nanp[threadIdx.x >> 6] = nn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float l = ((part[0] + part[1]) + (part[2] + part[3])) * inv_div;
    loss[0] = l;
    if (acc.loss_sum) {
      acc.loss_sum[0] = __fadd_rn(acc.loss_sum[0], __fmul_rn(l, acc.scale));
      acc.nan_count[0] += ((nanp[0] + nanp[1]) + (nanp[2] + nanp[3])) > 0.f ? 1 : 0;
      acc.steps[0] += 1;
    }
  }
  if (acc.d_pred) {  // the backward's d_pred for the promised upstream gradient (k_l1_bwd's formula)
    const float g = acc.d_loss[0] * inv_div;
    const int64_t nt = acc.rows_total * cols;
    for (int64_t e = threadIdx.x; e < nt; e += 256) {
      const int64_t i = e / cols, t = e - i * cols;
      float v = 0.f;
      if (i < rows) {
        const float d = p[i * ldp + t] - y[i * ldy + t];
        const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        v = sg * (w ? w[t] : 1.f) * g;
      }
      acc.d_pred[i * acc.ldd + t] = v;
    }
  }
}

__global__ void k_l1_bwd(const float* __restrict__ p, int64_t ldp, const float* __restrict__ y, int64_t ldy,
                         int64_t rows, int64_t cols, const float* __restrict__ w, float inv_div,
                         const float* __restrict__ dloss, float* __restrict__ dp, int64_t ldd, int64_t rows_total) {
  const int64_t n = rows_total * cols;
  const float g = dloss[0] * inv_div;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / cols, t = e - i * cols;
    if (i >= rows) {  // rows past the loss's rows (padding): zero gradient
      dp[i * ldd + t] = 0.f;
      continue;
    }
    const float d = p[i * ldp + t] - y[i * ldy + t];
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    dp[i * ldd + t] = sg * (w ? w[t] : 1.f) * g;
  }
}

}  // namespace
}  // namespace aimx

using namespace aimx;

extern "C" int aimx_l1_loss_forward_accum(const float* pred, int64_t ldp, const float* target, int64_t ldt,
                                          int64_t rows, int64_t cols, const float* weights, int32_t per_sample,
                                          float* loss, const AimxLossAccum* accum, aimx_stream_t stream) {
  if (rows < 0 || cols < 0 || !loss || ldp < cols || ldt < cols) return AIMX_EARG;
  if (rows * cols > 0 && (!pred || !target)) return AIMX_EARG;
  AimxLossAccum acc{};
  if (accum) {
    if (!accum->loss_sum || !accum->nan_count || !accum->steps) return AIMX_EARG;
    if (accum->d_pred && (!accum->d_loss || accum->ldd < cols || accum->rows_total < rows)) return AIMX_EARG;
    acc = *accum;
  }
  const double div = per_sample ? (double)rows : (double)rows * (double)cols;
  const float inv = div > 0 ? (float)(1.0 / div) : __builtin_nanf("");  // mean of nothing: NaN, as ATen
  hipLaunchKernelGGL(k_l1_fwd, dim3(1), dim3(256), 0, (hipStream_t)stream, pred, ldp, target, ldt, rows, cols, weights,
                     inv, loss, acc);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_l1_loss_forward(const float* pred, int64_t ldp, const float* target, int64_t ldt, int64_t rows,
                                    int64_t cols, const float* weights, int32_t per_sample, float* loss,
                                    aimx_stream_t stream) {
  return aimx_l1_loss_forward_accum(pred, ldp, target, ldt, rows, cols, weights, per_sample, loss, nullptr, stream);
}

extern "C" int aimx_l1_loss_backward_padded(const float* pred, int64_t ldp, const float* target, int64_t ldt,
                                            int64_t rows, int64_t rows_total, int64_t cols, const float* weights,
                                            int32_t per_sample, const float* d_loss, float* d_pred, int64_t ldd,
                                            aimx_stream_t stream) {
  if (rows < 0 || rows_total < rows || cols < 0 || ldp < cols || ldt < cols || ldd < cols || !d_loss) return AIMX_EARG;
  if (rows_total * cols == 0) return AIMX_OK;
  if ((rows > 0 && (!pred || !target)) || !d_pred) return AIMX_EARG;
  const double div = per_sample ? (double)rows : (double)rows * (double)cols;
  const int64_t blocks = std::min<int64_t>(cdiv(rows_total * cols, 256), 1024);
  hipLaunchKernelGGL(k_l1_bwd, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, pred, ldp, target, ldt, rows,
                     cols, weights, (float)(1.0 / div), d_loss, d_pred, ldd, rows_total);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

extern "C" int aimx_l1_loss_backward(const float* pred, int64_t ldp, const float* target, int64_t ldt, int64_t rows,
                                     int64_t cols, const float* weights, int32_t per_sample, const float* d_loss,
                                     float* d_pred, int64_t ldd, aimx_stream_t stream) {
  return aimx_l1_loss_backward_padded(pred, ldp, target, ldt, rows, rows, cols, weights, per_sample, d_loss, d_pred,
                                      ldd, stream);
}
