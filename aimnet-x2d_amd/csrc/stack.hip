// Message-passing stack orchestration (host side of the C ABI): one call enqueues a whole
// GNN._message_passing_forward (reference src/models/gnn.py:276-308) — per layer the partial
// charges (gnn.py:622-658), the hop (layers.py:133-167) written straight into the column chunks
// of the concatenated feature matrix F (layers.py:76-79, no cat), and the node-update MLP
// (layers.py:82-106) as five fused MFMA GEMMs whose epilogues carry bias, activation, dropout,
// the per-block residual, the global skip and the outer residual (gnn.py:302-306). The next
// layer's input is written by the last GEMM directly into chunk 0 of the next layer's F.
// The backward replays the same structure in reverse with fused act'/dropout epilogues and the
// hop backward as the same segmented gather-sum over the src-keyed CSR with the two residual
// terms fused; the activation gradients every weight gradient needs are kept, and all weight and
// bias gradients of the stack run at the end as ONE grouped launch (aimx_wgrad_grouped).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aimx_common.h"

namespace aimx {
namespace {

#define RUN(expr)                 \
  do {                            \
    int _r = (expr);              \
    if (_r != AIMX_OK) return _r; \
  } while (0)

AimxGemmArgs gemm0() {
  AimxGemmArgs a;
  memset(&a, 0, sizeof(a));
  a.act = ACT_NONE;
  a.dact_kind = ACT_NONE;
  return a;
}

// C[M=rows, N=out] = X[rows, in] (ld ldx) . W[out, in]^T  (nn.Linear forward)
AimxGemmArgs linear_fwd(int64_t rows, int64_t in, int64_t out, const float* X, int64_t ldx, const float* W,
                        float* C, int64_t ldc) {
  AimxGemmArgs a = gemm0();
  a.M = rows;
  a.N = out;
  a.K = in;
  a.A = X;
  a.sam = ldx;
  a.sak = 1;
  a.B = W;
  a.sbk = 1;
  a.sbn = in;
  a.C = C;
  a.ldc = ldc;
  return a;
}

// C[rows, in] = dY[rows, out] (ld) . W[out, in]  (input gradient)
AimxGemmArgs linear_dx(int64_t rows, int64_t in, int64_t out, const float* dY, int64_t ldy, const float* W, float* C,
                       int64_t ldc) {
  AimxGemmArgs a = gemm0();
  a.M = rows;
  a.N = in;
  a.K = out;
  a.A = dY;
  a.sam = ldy;
  a.sak = 1;
  a.B = W;
  a.sbk = in;
  a.sbn = 1;
  a.C = C;
  a.ldc = ldc;
  return a;
}

// dW[out, in] = dY^T . X, db[out] = sum_rows dY  (weight + bias gradient, K = rows)
AimxGemmArgs linear_dw(int64_t rows, int64_t in, int64_t out, const float* dY, int64_t ldy, const float* X,
                       int64_t ldx, float* dW, float* db) {
  AimxGemmArgs a = gemm0();
  a.M = out;
  a.N = in + 1;
  a.K = rows;
  a.A = dY;
  a.sam = 1;
  a.sak = ldy;
  a.B = X;
  a.sbk = ldx;
  a.sbn = 1;
  a.C = dW;
  a.ldc = in;
  a.ones_col = 1;
  a.col_out = db;
  return a;
}

// Strided 2-D copy as a kernel: dst[r*ldd + c] = src[r*lds + c]. (hipMemcpy2DAsync D2D nodes
// crashed the HIP runtime at stream-capture end on ROCm 7.2; a kernel node is also cheaper.)
// Rows go to workgroups (grid-stride), columns to threads: no per-element division (the flat-index
// form spent most of its 9.3 us on 64-bit div/mod at c5's 10 k x 307).
__global__ void k_copy2d(const float* __restrict__ src, int64_t lds, float* __restrict__ dst, int64_t ldd,
                         int64_t rows, int64_t cols) {
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x)
    for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) dst[r * ldd + c] = src[r * lds + c];
}

int copy2d(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t rows, int64_t cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return AIMX_OK;
  const int64_t blocks = std::min<int64_t>(rows, 8192);
  hipLaunchKernelGGL(k_copy2d, dim3((unsigned)blocks), dim3(cols > 128 ? 256 : 128), 0, s, src, lds, dst, ldd, rows, cols);
  AIMX_CHECK_LAUNCH();
  return AIMX_OK;
}

// A shell layer without MLP blocks (shell_conv_num_mlp_layers = 0: cli.py:106-107 accepts it):
// out = act(u) + g (layers.py:82-89, 106), + the outer residual x when stacked (gnn.py:302-306),
// added in the reference's order. UG = [act(u) | g] (row stride 2D).
__global__ void k_nomlp_fwd(const float* __restrict__ UG, int64_t ldug, int64_t D, const float* __restrict__ res,
                            int64_t ldr, float* __restrict__ dst, int64_t ldd, int64_t N) {
  const int64_t total = N * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D, c = i - r * D;
    float v = UG[r * ldug + c] + UG[r * ldug + D + c];
    if (res) v = v + res[r * ldr + c];
    dst[r * ldd + c] = v;
  }
}

// Its backward: dUG = [dY * act'(u) | dY] (U = the saved pre-activation u). dY may be dUG's own
// upper half (below the top layer the hop backward wrote it there): then only du is written.
__global__ void k_nomlp_bwd(const float* __restrict__ dY, int64_t ldy, const float* __restrict__ U, int act,
                            float* __restrict__ dUG, int64_t ldug, int64_t N, int64_t D, int copy_dy) {
  const int64_t total = N * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D, c = i - r * D;
    const float y = dY[r * ldy + c];
    dUG[r * ldug + c] = y * act_grad(act, U[r * D + c]);
    if (copy_dy) dUG[r * ldug + D + c] = y;
  }
}

int nomlp_blocks(int64_t N, int64_t D) { return (int)std::min<int64_t>(cdiv(N * D, 256), 8192); }

struct Ws {
  float* p;
  size_t bytes;
  int32_t* counters;
  int64_t n_counters;
  int32_t precision;
};

int run(AimxGemmArgs a, const Ws& ws, hipStream_t s) {
  a.workspace = ws.p;
  a.workspace_bytes = ws.bytes;
  a.counters = ws.counters;
  a.n_counters = ws.n_counters;
  a.precision = ws.precision;
  return launch_gemm(a, s);
}

int gather(const AimxShellStack* st, const float* src, int64_t src_ld, int64_t src_rpc, int64_t src_cs, int64_t D,
           const int32_t* rowptr, const int32_t* col, int64_t rows, float* out, int64_t out_ld, int64_t out_rpc,
           int64_t out_cs, const float* add0, int64_t add0_ld, const float* add1, int64_t add1_ld, hipStream_t s,
           int32_t skip_tail = 0) {
  return segment_gather_sum(src, src_ld, src_rpc, src_cs, D, rowptr, col, rows, out, out_ld, out_rpc, out_cs, add0,
                            add0_ld, add1, add1_ld, st->row_seg, st->row_seg_stride, s, skip_tail);
}

// Empty hop chunks (AimxGemmArgs.zc_*): every GEMM over F's columns trims the all-zero chunks the
// reference's hop leaves (layers.py:154), detected on the device from the forward CSR row pointers.
bool zc_on() { return tune_i64("AIMX_NO_ZC", 0) == 0; }  // tuning build: AIMX_NO_ZC=1 disables it

void set_zc(AimxGemmArgs& a, const AimxShellStack* s, int dim) {
  if (!zc_on() || !s->fwd_rowptr) return;
  a.zc_rowptr = s->fwd_rowptr;
  a.zc_rows = s->N;
  a.zc_chunks = (int32_t)s->num_hops;
  a.zc_width = s->D;
  a.zc_dim = dim;
}

bool valid(const AimxShellStack* s) {
  if (!s || s->N < 0 || s->D < 1 || s->num_hops < 1 || s->num_layers < 1 || s->num_mlp < 0) return false;
  if (s->ld_f < 0 || s->ld_ug < 0 || s->ld_act < 0 || (s->ld_f > 0 && s->ld_f < s->D * (s->num_hops + 1)) ||
      (s->ld_ug > 0 && s->ld_ug < 2 * s->D) || (s->ld_act > 0 && s->ld_act < s->D))
    return false;
  if (s->mode_single && (s->num_layers != 1 || s->use_pc)) return false;
  if (s->use_pc && (s->D < 2 || !s->gptr || !s->gperm || !s->total_charges)) return false;
  return true;
}


}  // namespace
}  // namespace aimx

using namespace aimx;

namespace aimx {
namespace {
// floats of the forward workspace's split-K region; the MLP weight images (mlp.hip) follow it
size_t fwd_split_floats(const AimxShellStack* s) {
  const int64_t N = s->N, D = s->D, K = D * (s->num_hops + 1);
  size_t need = 0;
  // The largest split-K products: weight gradients with K = N rows.
  AimxGemmArgs a = linear_dw(N, K, 2 * D, nullptr, 2 * D, nullptr, K, nullptr, nullptr);
  need = std::max(need, gemm_workspace_floats(a));
  a = linear_dw(N, D, D, nullptr, D, nullptr, D, nullptr, nullptr);
  need = std::max(need, gemm_workspace_floats(a));
  a = linear_fwd(N, K, 2 * D, nullptr, K, nullptr, nullptr, 2 * D);
  need = std::max(need, gemm_workspace_floats(a));
  a = linear_dx(N, K, 2 * D, nullptr, 2 * D, nullptr, nullptr, K);
  need = std::max(need, gemm_workspace_floats(a));
  return (need + 63) / 64 * 64;
}
}  // namespace
}  // namespace aimx

extern "C" size_t aimx_shell_stack_workspace_bytes(const AimxShellStack* s) {
  if (!valid(s)) return 0;
  return sizeof(float) * (fwd_split_floats(s) + mlp_pack_floats(s)) + 256;
}

extern "C" int aimx_shell_stack_forward(const AimxShellStack* s, aimx_stream_t stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (!valid(s)) return AIMX_EARG;
  const int64_t N = s->N, D = s->D, h = s->num_hops, L = s->num_layers, nm = s->num_mlp;
  const int64_t K = D * (h + 1), D2 = 2 * D;
  const int64_t LF = stack_ld_f(s), LUG = stack_ld_ug(s), LA = stack_ld_act(s);  // F / UG / R, A row strides
  if (N == 0) return AIMX_OK;
  const size_t split = fwd_split_floats(s), npack = mlp_pack_floats(s);
  float* pack = nullptr;
  if (npack) {  // the MLP weights as MFMA-fragment images, once for all layers (weight-streamed MLP)
    if (!s->workspace || s->workspace_bytes < sizeof(float) * (split + npack)) return AIMX_EARG;
    pack = s->workspace + split;
    RUN(launch_mlp_pack(s, false, pack, st));
  }
  const Ws ws{s->workspace, npack ? sizeof(float) * split : s->workspace_bytes, s->counters, s->n_counters,
              s->precision};
  const bool drop = s->training && s->drop_p > 0.f;
  for (int64_t l = 0; l < L; ++l) {
    float* F = s->F[l];
    // 1) layer input -> chunk 0 of F (after partial charges when enabled)
    if (s->use_pc) {
      const float* raw = (l == 0) ? s->x_in : s->X[l];
      const int64_t ldr = (l == 0) ? s->x_in_ld : D;
      RUN(launch_charge_fwd(raw, ldr, N, D, s->gptr, s->gperm, s->G, s->total_charges, F, LF, st));
    } else if (l == 0) {
      RUN(copy2d(s->x_in, s->x_in_ld, F, LF, N, D, st));
    }
    // 2) hop: chunks 1..h of F = scatter_add(x[src % N], target) in edge order. The trailing
    //    edge-less chunks (all but the first for reference inputs, layers.py:154) are not written:
    //    every GEMM over F trims them exactly (zc_*: the input projection's k loop stops before
    //    them, the weight gradient reads them as zero), so their zeros would be dead stores
    RUN(gather(s, F, LF, 0, 0, D, s->fwd_rowptr, s->fwd_col, N * h, F + D, LF, N, D, nullptr, 0, nullptr, 0, st,
               zc_on() ? 1 : 0));
    // 3) [u | g] = F [Wi ; Wg]^T + [bi ; bg], a0 = act(u)
    {
      AimxGemmArgs a = linear_fwd(N, K, D2, F, LF, s->w_ig[l], s->UG[l], LUG);
      set_zc(a, s, 0);
      a.bias = s->b_ig[l];
      a.act = s->act;
      a.act_ncols = D;
      a.pre = s->U[l];
      a.ldpre = D;
      RUN(run(a, ws, st));
    }
    // 4) MLP blocks: one fused launch for all of them (mlp.hip), or one GEMM per linear
    if (nm == 0) {  // no blocks: out = act(u) + g (+ x)
      float* dst = (l == L - 1) ? s->out : s->use_pc ? s->X[l + 1] : s->F[l + 1];
      const int64_t ldd = (l == L - 1) ? s->out_ld : s->use_pc ? D : LF;
      hipLaunchKernelGGL(k_nomlp_fwd, dim3((unsigned)nomlp_blocks(N, D)), dim3(256), 0, st, s->UG[l], LUG, D,
                         s->mode_single ? nullptr : F, LF, dst, ldd, N);
      AIMX_CHECK_LAUNCH();
      continue;
    }
    if (mlp_fused_ok(N, D, nm, s->precision, std::max({LF, LUG, LA, s->out_ld}))) {
      float* dst;
      int64_t ldd;
      if (l == L - 1) {
        dst = s->out;
        ldd = s->out_ld;
      } else if (s->use_pc) {
        dst = s->X[l + 1];
        ldd = D;
      } else {
        dst = s->F[l + 1];
        ldd = LF;
      }
      RUN(launch_mlp_fwd(s, l, s->mode_single ? nullptr : F, LF, dst, ldd, pack, st));
      continue;
    }
    for (int64_t k = 0; k < nm; ++k) {
      const int64_t idx = l * nm + k;
      const float* in = (k == 0) ? s->UG[l] : s->A[idx - 1];
      const int64_t ldin = (k == 0) ? LUG : LA;
      {
        AimxGemmArgs a = linear_fwd(N, D, D, in, ldin, s->w1[idx], s->R[idx], LA);
        a.bias = s->b1[idx];
        a.act = s->act;
        a.act_ncols = D;
        a.pre = s->V[idx];
        a.ldpre = D;
        if (drop) {
          a.drop_p = s->drop_p;
          a.drop_seed = s->drop_seed;
          a.drop_salt = (uint32_t)idx;
          a.mask_out = s->M[idx];
          a.ldmask = D;
        }
        RUN(run(a, ws, st));
      }
      {
        const bool last = (k == nm - 1);
        float* dst;
        int64_t ldd;
        if (!last) {
          dst = s->A[idx];
          ldd = LA;
        } else if (l == L - 1) {
          dst = s->out;
          ldd = s->out_ld;
        } else if (s->use_pc) {
          dst = s->X[l + 1];
          ldd = D;
        } else {
          dst = s->F[l + 1];
          ldd = LF;
        }
        AimxGemmArgs a = linear_fwd(N, D, D, s->R[idx], LA, s->w2[idx], dst, ldd);
        a.bias = s->b2[idx];
        a.res[0] = in;  // per-block skip (layers.py:103)
        a.ldres[0] = ldin;
        if (last) {
          a.res[1] = s->UG[l] + D;  // global skip (layers.py:106)
          a.ldres[1] = LUG;
          if (!s->mode_single) {
            a.res[2] = F;  // outer residual x (gnn.py:302-306), after partial charges
            a.ldres[2] = LF;
          }
        }
        RUN(run(a, ws, st));
      }
    }
  }
  return AIMX_OK;
}

namespace aimx {
namespace {

// Backward scratch layout (floats, 64-aligned regions); every gradient a weight gradient needs
// stays live until the grouped launch at the end.
struct BwdLayout {
  int64_t dF, dUG, dV, dA, dY, T0, pk, wg, total;  // offsets (floats); pk: MLP weight images (0 floats
                                                    // unless weight-streamed); wg: grouped-wgrad workspace
  int64_t nA, nY;
};

int64_t al64(int64_t x) { return (x + 63) / 64 * 64; }

// The top layer's upstream gradient as the stack reads it: an external view whose rows are not
// 16-byte aligned (c5: the x_other columns of the concat's input gradient) is copied once into the
// dY slot of layer L-1 (16-byte rows), so the weight gradient of its last MLP block does not force
// the grouped launch onto its per-problem load path.
bool top_dy_copied(const AimxShellStack* s, const AimxShellStackGrad* g) {
  return stack_ld_act(s) % 4 == 0 && g->d_out && ((g->d_out_ld % 4) != 0 || ((uintptr_t)g->d_out & 15) != 0);
}

// one AimxWgradProblem per weight gradient of the stack, in launch order
int stack_wgrad_problems(const AimxShellStack* s, const AimxShellStackGrad* g, const float* base, const BwdLayout* L_,
                         AimxWgradProblem* out) {
  const int64_t N = s->N, D = s->D, h = s->num_hops, L = s->num_layers, nm = s->num_mlp;
  const int64_t K = D * (h + 1), D2 = 2 * D;
  const int64_t LF = stack_ld_f(s), LUG = stack_ld_ug(s), LA = stack_ld_act(s);
  int n = 0;
  for (int64_t l = L - 1; l >= 0; --l) {
    const float* dYl = nullptr;
    int64_t ldy = D;
    if (base) {  // below the top layer, dY is the hop backward's output (its own 16-byte rows)
      const bool ext = l == L - 1 && !top_dy_copied(s, g);
      dYl = ext ? g->d_out : base + L_->dY + l * N * LA;
      ldy = ext ? g->d_out_ld : LA;
    }
    for (int64_t k = nm - 1; k >= 0; --k) {
      const int64_t idx = l * nm + k;
      const float* da = (k == nm - 1) ? dYl : (base ? base + L_->dA + (l * (nm - 1) + k) * N * LA : nullptr);
      const int64_t lda = (k == nm - 1) ? ldy : LA;
      AimxWgradProblem w2 = {da, lda, base ? s->R[idx] : nullptr, LA, g ? g->d_w2[idx] : nullptr, D,
                             g ? g->d_b2[idx] : nullptr, D, D, N};
      const float* in = base ? ((k == 0) ? s->UG[l] : s->A[idx - 1]) : nullptr;
      AimxWgradProblem w1 = {base ? base + L_->dV + idx * N * LA : nullptr, LA, in, (k == 0) ? LUG : LA,
                             g ? g->d_w1[idx] : nullptr, D, g ? g->d_b1[idx] : nullptr, D, D, N};
      out[n++] = w2;
      out[n++] = w1;
    }
    AimxWgradProblem wig = {base ? base + L_->dUG + l * N * LUG : nullptr, LUG, base ? s->F[l] : nullptr, LF,
                            g ? g->d_w_ig[l] : nullptr, K, g ? g->d_b_ig[l] : nullptr, D2, K, N};
    if (zc_on() && s->fwd_rowptr) {  // weight columns of empty chunks get an exact zero gradient
      wig.zc_rowptr = s->fwd_rowptr;
      wig.zc_rows = N;
      wig.zc_chunks = (int32_t)h;
      wig.zc_width = D;
    }
    out[n++] = wig;
  }
  return n;
}

BwdLayout bwd_layout(const AimxShellStack* s) {
  const int64_t N = s->N, D = s->D, L = s->num_layers, nm = s->num_mlp;
  BwdLayout b;
  b.nA = L * (nm - 1);
  b.nY = L;  // layers 0..L-2: the hop backward's output; L-1: top_dy's aligned copy
  int64_t o = 0;
  b.dF = o, o += al64(N * stack_ld_f(s));
  b.dUG = o, o += al64(L * N * stack_ld_ug(s));
  b.dV = o, o += al64(L * nm * N * stack_ld_act(s));
  b.dA = o, o += al64(std::max<int64_t>(b.nA, 1) * N * stack_ld_act(s));
  b.dY = o, o += al64(std::max<int64_t>(b.nY, 1) * N * stack_ld_act(s));
  b.T0 = o, o += al64(N * D);
  b.pk = o, o += al64((int64_t)mlp_pack_floats(s));
  b.wg = o;
  // problem shapes only (null pointers, non-null col_out flags) for the grouped workspace size
  std::vector<AimxWgradProblem> pr(L * (2 * nm + 1));
  const int n = stack_wgrad_problems(s, nullptr, nullptr, &b, pr.data());
  for (int i = 0; i < n; ++i) pr[i].col_out = reinterpret_cast<float*>(16);
  o += al64((int64_t)(aimx_wgrad_grouped_workspace_bytes(pr.data(), n) / sizeof(float)));
  b.total = o;
  return b;
}

}  // namespace
}  // namespace aimx

extern "C" size_t aimx_shell_stack_backward_workspace_bytes(const AimxShellStack* s) {
  if (!valid(s)) return 0;
  return sizeof(float) * (size_t)bwd_layout(s).total + 256;
}

extern "C" int aimx_shell_stack_backward(const AimxShellStack* s, const AimxShellStackGrad* g, aimx_stream_t stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (!valid(s) || !g) return AIMX_EARG;
  const int64_t N = s->N, D = s->D, h = s->num_hops, L = s->num_layers, nm = s->num_mlp;
  const int64_t K = D * (h + 1), D2 = 2 * D;
  const int64_t LF = stack_ld_f(s), LUG = stack_ld_ug(s), LA = stack_ld_act(s);
  if (N == 0) return AIMX_OK;
  const BwdLayout lay = bwd_layout(s);
  if (!g->workspace || g->workspace_bytes < sizeof(float) * (size_t)lay.total) return AIMX_EARG;
  float* base = (float*)g->workspace;
  float* dF = base + lay.dF;
  // weight-gradient problems of the whole stack (layer L-1 first, 2*nm+1 per layer)
  const int per_layer = (int)(2 * nm + 1);
  std::vector<AimxWgradProblem> pr(L * per_layer);
  const int n_pr = stack_wgrad_problems(s, g, base, &lay, pr.data());
  const Ws ws{s->workspace, s->workspace_bytes, s->counters, s->n_counters, s->precision};
  float* wg_ws = base + lay.wg;
  const size_t wg_bytes = sizeof(float) * (size_t)(lay.total - lay.wg);
  const bool drop = s->training && s->drop_p > 0.f;
  float* pack = nullptr;
  if (mlp_pack_floats(s)) {  // transposed MLP weight images for the weight-streamed chain
    pack = base + lay.pk;
    RUN(launch_mlp_pack(s, true, pack, st));
  }
  if (top_dy_copied(s, g)) RUN(copy2d(g->d_out, g->d_out_ld, base + lay.dY + (L - 1) * N * LA, LA, N, D, st));
  for (int64_t l = L - 1; l >= 0; --l) {
    // dUG = [du | dg] with dg = dY. dY: the upstream gradient (top layer) or the hop backward's
    // output of layer l + 1, in a buffer of its own with 16-byte rows (the weight gradient of the
    // last MLP block reads it with 16-byte loads; dUG's upper half starts at the odd offset D); the
    // MLP chain copies it into dUG's upper half as it stages it
    float* dUG = base + lay.dUG + l * N * LUG;
    const bool ext = l == L - 1 && !top_dy_copied(s, g);
    const float* dY = ext ? g->d_out : base + lay.dY + l * N * LA;
    const int64_t ldy = ext ? g->d_out_ld : LA;
    // MLP blocks, last to first: only the activation-gradient chain here (weights deferred)
    const bool fused = nm > 0 && mlp_fused_ok(N, D, nm, s->precision, std::max({LF, LUG, LA, s->out_ld, g->d_out_ld}));
    if (nm == 0) {  // no blocks: dUG = [dY * act'(u) | dY]
      hipLaunchKernelGGL(k_nomlp_bwd, dim3((unsigned)nomlp_blocks(N, D)), dim3(256), 0, st, dY, ldy, s->U[l], s->act,
                         dUG, LUG, N, D, dY != dUG + D ? 1 : 0);
      AIMX_CHECK_LAUNCH();
    }
    if (fused) {  // the whole chain + dUG = [du | dY] in one launch (mlp.hip)
      float* dVs[8];
      float* dAs[8];
      for (int64_t k = 0; k < nm; ++k) {
        dVs[k] = base + lay.dV + (l * nm + k) * N * LA;
        dAs[k] = (k < nm - 1) ? base + lay.dA + (l * (nm - 1) + k) * N * LA : nullptr;
      }
      RUN(launch_mlp_bwd(s, l, dY, ldy, dVs, dAs, dUG, pack, st));
    }
    for (int64_t k = nm - 1; k >= 0 && !fused; --k) {
      const int64_t idx = l * nm + k;
      const float* da_out = (k == nm - 1) ? dY : base + lay.dA + (l * (nm - 1) + k) * N * LA;
      const int64_t ld_out = (k == nm - 1) ? ldy : LA;
      float* dV = base + lay.dV + idx * N * LA;
      {  // dV = (da_out W2) * mask/(1-p) * act'(V)
        AimxGemmArgs a = linear_dx(N, D, D, da_out, ld_out, s->w2[idx], dV, LA);
        if (drop) {
          a.drop_p = s->drop_p;
          a.mask_in = s->M[idx];
          a.ldmask = D;
        }
        a.dact_pre = s->V[idx];
        a.lddact = D;
        a.dact_kind = s->act;
        RUN(run(a, ws, st));
      }
      {  // da_in = da_out + dV W1 ; for k == 0 also * act'(u) -> du into dUG[:, :D]
        float* dst = (k == 0) ? dUG : base + lay.dA + (l * (nm - 1) + k - 1) * N * LA;
        const int64_t ldd = (k == 0) ? LUG : LA;
        AimxGemmArgs a = linear_dx(N, D, D, dV, LA, s->w1[idx], dst, ldd);
        a.res[0] = da_out;
        a.ldres[0] = ld_out;
        if (k == 0) {
          a.dact_pre = s->U[l];
          a.lddact = D;
          a.dact_kind = s->act;
        }
        RUN(run(a, ws, st));
      }
    }
    // dg = dY -> dUG[:, D:] (the fused chain writes it itself)
    if (!fused && nm > 0 && dY != dUG + D) RUN(copy2d(dY, ldy, dUG + D, LUG, N, D, st));
    {  // dF = dUG [Wi ; Wg]; tiles wholly in the trailing empty chunks are not computed nor stored:
       // the hop backward gathers only from chunks that hold targets (zc_dim 2)
      AimxGemmArgs a = linear_dx(N, K, D2, dUG, LUG, s->w_ig[l], dF, LF);
      set_zc(a, s, 2);
      RUN(run(a, ws, st));
    }
    // hop backward + chunk-0 gradient + outer residual: dx = dF[:, :D] + dY + sum_{e: src%N == j} dF_agg[target_e]
    const bool first = (l == 0);
    float* nxt = first ? g->d_x_in : base + lay.dY + (l - 1) * N * LA;  // layer l-1's dY
    const int64_t ldn = first ? g->d_x_in_ld : LA;
    float* dst = s->use_pc ? base + lay.T0 : nxt;
    const int64_t ldd = s->use_pc ? D : ldn;
    RUN(gather(s, dF + D, LF, N, D, D, s->bwd_rowptr, s->bwd_col, N, dst, ldd, 0, 0, dF, LF,
               s->mode_single ? nullptr : dY, ldy, st));
    if (s->use_pc) {
      const float* raw = first ? s->x_in : s->X[l];
      const int64_t ldr = first ? s->x_in_ld : D;
      RUN(launch_charge_bwd(raw, ldr, N, D, s->gptr, s->gperm, s->G, s->total_charges, dst, D, nxt, ldn, st));
    }
  }
  // every weight and bias gradient of the stack in one grouped launch
  return aimx_wgrad_grouped(pr.data(), n_pr, wg_ws, wg_bytes, s->counters, s->n_counters, stream_);
}
