/*
 * aimx.h — C ABI of the MI355X-native AIMNet-X2D message-passing / attention-pool hot path.
 *
 * Library: aimnet-x2d_amd/lib/libaimx.so (HIP, gfx950). Plain pointers and sizes only; every
 * device pointer is a HIP device allocation owned by the caller (the PyTorch caching allocator in
 * the Python mirror), and every call only ENQUEUES work on `stream` (a hipStream_t): no host
 * synchronisation, no allocation, no global mutable state. Functions return 0 on success, a
 * hipError_t value (> 0) if a HIP call failed, or AIMX_EARG (< 0) on invalid arguments.
 *
 * The reference (mahdi-shafiei/AIMNet-X2D) has no FFI: its hot path is pure PyTorch plus
 * torch_scatter. Each entry point below names the reference interface it replaces; the Python
 * mirror (aimnet-x2d_amd/models, aimnet-x2d_amd/utils) binds them with ctypes behind the
 * reference's own module API.
 */
#ifndef AIMX_H_
#define AIMX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* aimx_stream_t; /* hipStream_t */

#define AIMX_OK 0
#define AIMX_EARG (-1)

/* Status bits written (OR-ed) into the optional device `status` word. */
#define AIMX_STATUS_KEY_OUT_OF_RANGE 1 /* an index outside [0, n_rows): item dropped (reference raises) */

/* Activation kinds (reference src/utils/activation.py:9-34). */
#define AIMX_ACT_NONE (-1)
#define AIMX_ACT_RELU 0
#define AIMX_ACT_LEAKYRELU 1
#define AIMX_ACT_ELU 2
#define AIMX_ACT_GELU 3
#define AIMX_ACT_SILU 4

/* Library identity (for load checks): returns "aimx/<version>/gfx950". */
const char* aimx_version(void);

/* Path options: test hooks, not a tuning surface. The product library reads no environment
 * variable; every launcher uses its defaults unless an option of the same name was set here (the
 * alternative-path parity tests):
 *   "AIMX_MLPW"         0 = per-GEMM node-update MLP instead of the weight-resident kernels
 *   "AIMX_MLPS"         0 / 1 = weight-streamed MLP off / for every width
 *   "AIMX_MLPS_RT"      row tiles per chunk of the weight-streamed MLP
 *   "AIMX_WGRAD_BB"     64 / 80 = weight-gradient block edge
 *   "AIMX_GEMM_DEEP"    0 = few-row deep-K products on the LDS-staged tiles; 8 = 8 waves
 *   "AIMX_HOP_MAX_ROWS" n = the hop's row-range splitting at n rows per launch (not 2^31)
 * The tuning build (make tune -> lib/libaimx_tune.so) also reads these names, and its A/B knobs
 * (tune_i64 in csrc: variants measured slower, kept for re-measurement), from the environment; the
 * product library compiles those knobs to their defaults. aimx_set_option returns AIMX_EARG for a
 * name longer than 47 bytes or past 16 names. */
int aimx_set_option(const char* name, int64_t value);
int aimx_clear_options(void);

/* ------------------------------------------------------------------------------------------
 * Stable CSR build (device): rows sorted by key, ties kept in ascending item order — exactly the
 * order in which CPU ATen scatter_add_ visits edges (reference layers.py:158 via torch_scatter
 * scatter_add, and pooling.py:145/159 via scatter_softmax/scatter_sum). Replaces the implicit
 * COO->segment step inside torch_scatter.
 *   key(i) = key[i*key_stride], taken modulo key_mod (Python semantics) when key_mod > 0
 *   val(i) = val ? val[i*val_stride] (mod val_mod) : i
 *   rowptr[n_rows+1] (int32), col[n_items] (int32).
 * Items with key outside [0, n_rows) are dropped and AIMX_STATUS_KEY_OUT_OF_RANGE is OR-ed into
 * *status (if non-NULL) — the reference would raise an index error instead.
 * ------------------------------------------------------------------------------------------ */
size_t aimx_csr_workspace_bytes(int64_t n_items, int64_t n_rows);
int aimx_csr_build(const int64_t* key, int64_t key_stride, int64_t key_mod,
                   const int64_t* val, int64_t val_stride, int64_t val_mod,
                   int64_t n_items, int64_t n_rows, int32_t* rowptr, int32_t* col,
                   void* workspace, size_t workspace_bytes, int32_t* status, aimx_stream_t stream);

/* Several CSRs (at most 4) in one pass — one launch per phase for all of them. Each spec is the
 * argument set of aimx_csr_build; rowptr/col are written per spec exactly as aimx_csr_build
 * would (bit-identical), keys out of range are flagged in *status. *status is set to 0 first
 * (by the call's own zero-fill launch: the caller need not zero it; a status word is per call). */
typedef struct {
  const int64_t* key;
  int64_t key_stride, key_mod;
  const int64_t* val;
  int64_t val_stride, val_mod;
  int64_t n_items, n_rows;
  int32_t* rowptr;
  int32_t* col;
} AimxCsrSpec;

size_t aimx_csr_build_multi_workspace_bytes(const AimxCsrSpec* specs, int32_t n);
int aimx_csr_build_multi(const AimxCsrSpec* specs, int32_t n, void* workspace, size_t workspace_bytes,
                         int32_t* status, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Multi-hop scatter-add as a segmented gather-sum (the hop).
 * Replaces ShellConvolutionLayer.message_passing (reference src/models/layers.py:133-167):
 *   out[t,:] = sum over edges e with target_e == t of x[src_e % N, :], summed in edge order
 * (bit-exact with the reference forward). The same kernel is the backward of the hop over the
 * src-keyed CSR (grad_x[j] = sum over e with src_e % N == j of grad_out[target_e]).
 * Row addressing (src and out): row r lives at base + (r % rows_per_chunk)*ld
 * + (r / rows_per_chunk)*chunk_stride (rows_per_chunk <= 0: base + r*ld), so the output can be
 * written straight into the column chunks of the concatenated [N, D*(h+1)] feature matrix
 * (layers.py:76-79) without a cat. add0/add1 (nullable, indexed by output row, plain ld) are
 * added to each output row (fused residual terms in the backward). Output rows past the first
 * chunk are expected to be mostly edge-free (the reference's hop chunks >= 1) and are walked in
 * large tiles; pass out_rows_per_chunk = N, out_chunk_stride = N*out_ld for a plain [h*N, D]
 * output to get that (same addresses as rows_per_chunk <= 0).
 * row_seg (nullable, stride row_seg_stride): segment id per row of the first output chunk —
 * the molecule index (batch_indices) for the hop and its backward, whose rows are atoms. Rows
 * of one segment are consecutive and edges stay inside a segment, so row tiles cut at segment
 * starts (when one lies within 64 rows of the nominal cut) stage their source rows exactly once;
 * for rows that are not 16-byte vectors (odd D such as 153 / 307, or unaligned chunk offsets) a
 * tile is the set of whole segments that start in a window of rows. The result does not depend on
 * row_seg (it only moves tile boundaries). Rows must be 4-byte aligned (fp32).
 * ------------------------------------------------------------------------------------------ */
int aimx_segment_gather_sum(const float* src, int64_t src_ld, int64_t src_rows_per_chunk,
                            int64_t src_chunk_stride, int64_t D,
                            const int32_t* rowptr, const int32_t* col, int64_t rows,
                            float* out, int64_t out_ld, int64_t out_rows_per_chunk,
                            int64_t out_chunk_stride,
                            const float* add0, int64_t add0_ld, const float* add1, int64_t add1_ld,
                            const int64_t* row_seg, int64_t row_seg_stride, aimx_stream_t stream);

/* aimx_segment_gather_sum with flags. AIMX_GATHER_SKIP_TAIL: output chunks in the trailing run of
 * edge-less chunks (out_rows_per_chunk > 0) are NOT written — their rows keep whatever the buffer
 * held. For consumers that never read those chunks: the message-passing stack's hop (the reference's
 * chunks >= 1 are empty, layers.py:154, and its GEMMs trim them exactly, AimxGemmArgs.zc_*). The
 * call the stack makes per layer, exposed so that its cost can be timed on its own. */
#define AIMX_GATHER_SKIP_TAIL 1
int aimx_segment_gather_sum_ex(const float* src, int64_t src_ld, int64_t src_rows_per_chunk,
                               int64_t src_chunk_stride, int64_t D,
                               const int32_t* rowptr, const int32_t* col, int64_t rows,
                               float* out, int64_t out_ld, int64_t out_rows_per_chunk,
                               int64_t out_chunk_stride,
                               const float* add0, int64_t add0_ld, const float* add1, int64_t add1_ld,
                               const int64_t* row_seg, int64_t row_seg_stride, int32_t flags,
                               aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Fused fp32 GEMM on the matrix cores (v_mfma_f32_16x16x4_f32; exact f32 fmaf chains), the
 * building block of the node-update MLP (reference layers.py:82-106, nn.Linear/addmm):
 *   C(m,n) = epilogue( sum_k A(m,k) * B(k,n) )
 *   A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn]
 * Epilogue, in order: (+ beta*C_old) (+ bias[n]) (+ res0 + res1 + res2) (pre <- v for
 * n < act_ncols) (v = act(v) for n < act_ncols) (forward dropout with hash(seed, salt, m, n),
 * mask written to mask_out) (v *= mask_in ? 1/(1-p) : 0) (v *= act'(dact_pre)) -> C.
 * ones_col != 0: B gets an implicit all-ones column at n == N-1 and column N-1 of the result is
 * written to col_out[m] instead of C (bias gradient fused into the weight-gradient GEMM).
 * splits > 1 (0 = automatic): split-K with partial slabs in `workspace`, reduced in slab order
 * (deterministic) inside the launch when `counters` is given.
 * ------------------------------------------------------------------------------------------ */
typedef struct AimxGemmArgs {
  int64_t M, N, K;
  const float* A; int64_t sam, sak;
  const float* B; int64_t sbk, sbn;
  float* C; int64_t ldc;
  float beta;
  const float* bias;
  const float* res[3]; int64_t ldres[3];
  int32_t act; int64_t act_ncols;
  float* pre; int64_t ldpre;
  const float* dact_pre; int64_t lddact; int32_t dact_kind;
  float drop_p; const int64_t* drop_seed; uint32_t drop_salt;
  uint8_t* mask_out; const uint8_t* mask_in; int64_t ldmask;
  int32_t ones_col; float* col_out;
  int32_t splits; float* workspace; size_t workspace_bytes;
  /* split-K tile arrival counters: zero-initialised, persistent, self-resetting (the last
   * arriving slice of a tile reduces the slabs in order and rezeroes its counter). NULL: a
   * separate ordered reduce kernel is launched instead. */
  int32_t* counters; int64_t n_counters;
  /* Empty hop chunks. The reference's hop adds every hop's pairs to chunk 0 (targets < N,
   * layers.py:154), so chunks 1..h-1 of message_passing's output are all-zero for reference
   * inputs. When zc_rowptr != NULL (the hop's forward CSR row pointers) the kernel reads, on the
   * device, E = zc_width * (1 + c) with c = 1 + the last chunk j in [0, zc_chunks) that holds an
   * edge (zc_rowptr[(j+1)*zc_rows] > zc_rowptr[j*zc_rows]; c = 0 if none):
   *   zc_dim 0: operand entries with k >= E are zero, so the k loop stops at E;
   *   zc_dim 1: output columns >= E (ones column excluded) are zero: whole tiles there are
   *             written as 0 without loads or MFMA work (plain-store epilogue only);
   *   zc_dim 2: as 1, but whole tiles past E are not written at all (the caller never reads
   *             those columns: the stack's hop-chunk input gradient, whose empty chunks the hop
   *             backward never gathers).
   * Results are identical to the untrimmed product (only exact zeros are skipped). */
  const int32_t* zc_rowptr; int64_t zc_rows; int32_t zc_chunks; int64_t zc_width; int32_t zc_dim;
  /* AIMX_PREC_FP32 (0, the parity path): exact fp32 products (v_mfma_f32_16x16x4_f32).
   * AIMX_PREC_BF16 (1, the mixed-precision path of the reference's --mixed_precision, trainer.py:
   * 134/238): A and B rounded to bf16 (RNE) when staged, products accumulated in fp32
   * (v_mfma_f32_16x16x32_bf16); C, the epilogue and every other tensor stay fp32. Long-K
   * weight-gradient GEMMs (A m-contiguous, B n-contiguous, K >= 512) stay exact fp32. */
  int32_t precision;
  /* Row offset of this call's row 0 in a larger product (the dropout hash is keyed by the global row
   * m_base + m, so a product run as row chunks draws the masks of the one-launch product); 0 for a
   * caller's own calls. */
  int64_t m_base;
} AimxGemmArgs;
#define AIMX_PREC_FP32 0
#define AIMX_PREC_BF16 1

size_t aimx_gemm_workspace_bytes(const AimxGemmArgs* args);
int aimx_gemm(const AimxGemmArgs* args, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Message-passing stack: L x (partial charges?) -> ShellConvolutionLayer -> +x, fused.
 * Replaces GNN._message_passing_forward (reference src/models/gnn.py:276-308) with
 * ShellConvolutionLayer.forward (layers.py:63-108) and _partial_charge_calculation
 * (gnn.py:622-658). All activations are kept for the backward in caller-owned buffers:
 *   F[l]  [N, K=D*(h+1)]  concat features; column chunk 0 = layer input x_l (after charges)
 *   X[l]  [N, D]          raw layer input before partial charges (use_pc only)
 *   UG[l] [N, 2D]         [a0 | g] = [act(u) | global skip]       U[l] [N, D] = u (pre-act)
 *   V[l*nm+k], R[l*nm+k], A[l*nm+k] [N, D]  per MLP block: pre-act, dropped act, block output
 *   M[l*nm+k] [N, D] uint8 dropout masks (training && drop_p > 0)
 * w_ig[l] is the stacked [input_proj.weight ; global_skip_proj.weight] ([2D, K]), b_ig[l] [2D].
 * x_in [N, D] (ld x_in_ld) is the stack input; out [N, D] (ld out_ld) the output.
 * mode_single != 0 runs one ShellConvolutionLayer.forward without the outer residual and without
 * charges (the standalone layer API).
 * ------------------------------------------------------------------------------------------ */
typedef struct AimxShellStack {
  int64_t N, D, num_hops, num_layers, num_mlp;
  int32_t act, use_pc, training, mode_single;
  float drop_p; const int64_t* drop_seed;
  const int32_t* fwd_rowptr; const int32_t* fwd_col; /* rows N*num_hops, col = src % N */
  const int32_t* bwd_rowptr; const int32_t* bwd_col; /* rows N, col = target */
  const int32_t* gptr; const int32_t* gperm; int64_t G; const float* total_charges;
  const int64_t* row_seg; int64_t row_seg_stride; /* molecule id per atom (nullable): hop tiles */
  const float* const* w_ig; const float* const* b_ig;
  const float* const* w1; const float* const* b1; const float* const* w2; const float* const* b2;
  float* const* F; float* const* X; float* const* UG; float* const* U;
  float* const* V; float* const* R; float* const* A; uint8_t* const* M;
  const float* x_in; int64_t x_in_ld;
  float* out; int64_t out_ld;
  float* workspace; size_t workspace_bytes;
  int32_t* counters; int64_t n_counters; /* as in AimxGemmArgs */
  int32_t precision; /* AIMX_PREC_*: of the stack's node-update GEMMs (weight gradients stay fp32) */
  /* row strides (floats) of the F [N, D(h+1)] and UG [N, 2D] buffers and of their backward
   * counterparts (0: dense, K and 2D). Rounded up to 4 floats they make every row 16-byte aligned, so
   * the weight gradients over them take 16-byte loads at odd D (c4 / c5: D = 153 / 307) */
  int64_t ld_f, ld_ug;
  /* row stride of the R [N, D] and A [N, D] buffers (and of the backward's dV / dA): 0 = D */
  int64_t ld_act;
} AimxShellStack;

typedef struct AimxShellStackGrad {
  const float* d_out; int64_t d_out_ld;  /* grad w.r.t. out [N, D] */
  float* d_x_in; int64_t d_x_in_ld;      /* grad w.r.t. x_in (written) */
  float* const* d_w_ig; float* const* d_b_ig;   /* per layer [2D,K], [2D] (written) */
  float* const* d_w1; float* const* d_b1; float* const* d_w2; float* const* d_b2;
  /* scratch, caller-owned, aimx_shell_stack_backward_workspace_bytes(s) bytes: the per-layer /
   * per-block activation gradients are kept until the weight gradients of the whole stack run
   * as ONE grouped launch at the end (aimx_wgrad_grouped) */
  void* workspace; size_t workspace_bytes;
} AimxShellStackGrad;

size_t aimx_shell_stack_workspace_bytes(const AimxShellStack* s);
size_t aimx_shell_stack_backward_workspace_bytes(const AimxShellStack* s);
int aimx_shell_stack_forward(const AimxShellStack* s, aimx_stream_t stream);
int aimx_shell_stack_backward(const AimxShellStack* s, const AimxShellStackGrad* g,
                              aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Partial-charge equilibration (reference src/models/gnn.py:622-658), one molecule per
 * workgroup over the graph CSR (gptr [G+1], gperm [N]).
 * ------------------------------------------------------------------------------------------ */
int aimx_partial_charge_forward(const float* x, int64_t ldx, int64_t N, int64_t D,
                                const int32_t* gptr, const int32_t* gperm, int64_t G,
                                const float* total_charges, float* out, int64_t ldo,
                                aimx_stream_t stream);
int aimx_partial_charge_backward(const float* x, int64_t ldx, int64_t N, int64_t D,
                                 const int32_t* gptr, const int32_t* gperm, int64_t G,
                                 const float* total_charges, const float* d_out, int64_t ldd,
                                 float* d_x, int64_t lddx, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Multi-head attention graph pooling (reference src/models/pooling.py:122-172):
 *   s[h,n] = (x_n . W[h] + b[h]) / tau ; a = per-molecule softmax of s over its atoms (per head,
 *   torch_scatter.scatter_softmax) ; pooled[g] = mean_h sum_{n in g} a[h,n] x_n.
 * One workgroup per molecule. tau is a device scalar (the learnable temperature). scores [H,N]
 * is saved for the backward. The backward writes dx (every row), dW [H,C], db [H], dtau [1];
 * d_attn (nullable) is an upstream gradient on the returned attention weights.
 * ------------------------------------------------------------------------------------------ */
size_t aimx_attn_pool_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t G);
int aimx_attn_pool_forward(const float* x, int64_t ldx, int64_t N, int64_t C,
                           const float* W, const float* b, const float* tau, int64_t H,
                           const int32_t* gptr, const int32_t* gperm, int64_t G,
                           float* pooled, float* attn, float* scores, aimx_stream_t stream);
int aimx_attn_pool_backward(const float* x, int64_t ldx, int64_t N, int64_t C,
                            const float* W, const float* tau, int64_t H,
                            const int32_t* gptr, const int32_t* gperm, int64_t G,
                            const float* attn, const float* scores,
                            const float* d_pooled, const float* d_attn,
                            float* dx, int64_t lddx, float* dW, float* db, float* dtau,
                            void* workspace, size_t workspace_bytes, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Mean / max / sum graph pooling (reference src/models/pooling.py:15-80, torch_scatter
 * scatter_mean / scatter_max / scatter_add over molecules). kind: 0 = mean, 1 = max, 2 = sum.
 * max records the first arg-max atom per (molecule, channel) for the backward (empty molecule:
 * value 0, argmax = -1).
 * ------------------------------------------------------------------------------------------ */
int aimx_segment_pool_forward(int32_t kind, const float* x, int64_t ldx, int64_t N, int64_t C,
                              const int32_t* gptr, const int32_t* gperm, int64_t G,
                              float* out, int32_t* argmax, aimx_stream_t stream);
int aimx_segment_pool_backward(int32_t kind, const float* d_out, int64_t N, int64_t C,
                               const int32_t* gptr, const int32_t* gperm, int64_t G,
                               const int32_t* argmax, float* dx, int64_t lddx,
                               aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Atom-feature embeddings (reference src/models/gnn.py:262-274, nn.Embedding x4 + cat) and the
 * elementwise activation backward used around the dense projections.
 * gather:   out[j, t*dim + c] = table[t][index[t][j], c]            (out [N, n_tables*dim])
 * backward: grad[t] = sum over atoms j of dE[j, t*dim:(t+1)*dim] into row index[t][j]
 *           (deterministic: per-chunk partial tables in LDS, then an ordered reduce).
 * Indices are int64 (the reference's dtype); out-of-range indices contribute nothing.
 * ------------------------------------------------------------------------------------------ */
#define AIMX_MAX_TABLES 8
typedef struct AimxEmbeddingTables {
  int32_t n_tables; int64_t dim;
  const float* table[AIMX_MAX_TABLES];
  const int64_t* index[AIMX_MAX_TABLES];
  int64_t rows[AIMX_MAX_TABLES];
  float* grad[AIMX_MAX_TABLES];
  /* optional (n_seeds > 0, gather only): the gather launch also draws the forward's n_seeds
   * dropout seeds from the counter at seed_state, exactly as aimx_dropout_seeds would (one launch
   * fewer per step) */
  int64_t* seed_state;
  int64_t* seeds;
  int32_t n_seeds;
} AimxEmbeddingTables;

int aimx_embedding_gather(const AimxEmbeddingTables* t, int64_t N, float* out, int64_t ldo,
                          aimx_stream_t stream);
size_t aimx_embedding_backward_workspace_bytes(const AimxEmbeddingTables* t, int64_t N);
int aimx_embedding_backward(const AimxEmbeddingTables* t, int64_t N, const float* dE, int64_t ldd,
                            void* workspace, size_t workspace_bytes, aimx_stream_t stream);
/* out[m,n] = dy[m,n] * act'(pre[m,n]) */
int aimx_act_backward(int32_t kind, const float* dy, int64_t ldy, const float* pre, int64_t ldp,
                      int64_t M, int64_t N, float* out, int64_t ldo, aimx_stream_t stream);
/* The same over two column sources: dy[:, :n0] = dy0 (ld ldy0), dy[:, n0:] = dy1 (ld ldy1) — the
 * gradients of the x_self / x_other views of the embedding projection (gnn.py:227-231) in one
 * launch. Requires N, ldp, ldo % 4 == 0, 16-byte-aligned pre / out, 4-byte-aligned dy0 / dy1. */
int aimx_act_backward2(int32_t kind, const float* dy0, int64_t ldy0, int64_t n0, const float* dy1, int64_t ldy1,
                       const float* pre, int64_t ldp, int64_t M, int64_t N, float* out, int64_t ldo,
                       aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Grouped weight gradients: for each problem, dW[M, N] = dY^T X over K rows (atoms) and, when
 * col_out is non-NULL, col_out[M] = sum_k dY (the bias gradient) — the backward of nn.Linear's
 * weight and bias (reference layers.py:82-106 via autograd) for many layers in ONE launch.
 * dY is [K, M] row-major with row stride ld_dy, X is [K, N] with row stride ld_x. Deterministic
 * (fixed split-K order). Needs `counters` (>= sum of 32x32 tiles, kept zero by the kernel) and
 * aimx_wgrad_grouped_workspace_bytes() of workspace.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  const float* dY;
  int64_t ld_dy;
  const float* X;
  int64_t ld_x;
  float* dW;
  int64_t ld_dw;
  float* col_out;
  int64_t M, N, K;
  /* optional empty-chunk trimming of the N (= X column) dimension, as zc_dim 1 of AimxGemmArgs */
  const int32_t* zc_rowptr; int64_t zc_rows; int32_t zc_chunks; int64_t zc_width;
} AimxWgradProblem;

size_t aimx_wgrad_grouped_workspace_bytes(const AimxWgradProblem* problems, int32_t n);
int aimx_wgrad_grouped(const AimxWgradProblem* problems, int32_t n, void* workspace, size_t workspace_bytes,
                       int32_t* counters, int64_t n_counters, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Fused global-norm gradient clip + Adam step over a list of fp32 tensors (sum of squares and
 * update: one launch each per chunk of 80 tensors; one fold launch between them).
 * Replaces the trainer's  torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0);
 * optimizer.step()  with optimizer = torch.optim.Adam(...) (reference
 * src/training/trainer.py:163-164 and 221-223):
 *   total = ||all grads||_2; coef = min(max_norm / (total + 1e-6), 1) (max_norm <= 0: no clip);
 *   grad *= coef (in place); step[slot] += 1; [grad += weight_decay * param];
 *   exp_avg = lerp(exp_avg, grad, 1 - beta1); exp_avg_sq = beta2*exp_avg_sq + (1-beta2)*grad^2;
 *   param -= lr[group] / (1 - beta1^s) * exp_avg / (sqrt(exp_avg_sq) / sqrt(1 - beta2^s) + eps),
 *   s = step[slot]
 * `step` is an array of per-parameter step counters (torch.optim.Adam's state['step']): tensor i
 * advances and uses step[tensors[i].step_slot] (slots distinct within a call, < 2^23), so a
 * parameter left out of a step (no gradient) keeps its count, as in torch. `step` and `lr` (one
 * float per parameter group, group < 256) are device memory, so the call is graph-capturable and
 * schedulers update lr without re-capture. *norm_out (nullable, device) receives the total norm
 * clip_grad_norm_ returns. The workspace (aimx_fused_adam_workspace_bytes) holds the per-slice
 * partial sums of squares, folded by one workgroup in a fixed order into the clip coefficient
 * (deterministic, no arrival counter; zero-filling it is harmless, not needed).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
  int32_t group;
  int32_t step_slot;
} AimxAdamTensor;

/* one_minus_beta1/2 are passed separately because torch forms 1 - beta in double precision
 * (1 - 0.999f in fp32 is 1.3e-5 relative away from fp32(1 - 0.999)). */
typedef struct {
  float beta1, beta2, one_minus_beta1, one_minus_beta2, eps, weight_decay, max_grad_norm;
} AimxAdamHyper;

size_t aimx_fused_adam_workspace_bytes(const AimxAdamTensor* tensors, int32_t n);
int aimx_fused_adam(const AimxAdamTensor* tensors, int32_t n, const AimxAdamHyper* hyper, float* step,
                    const float* lr, float* norm_out, void* workspace, size_t workspace_bytes,
                    aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Fused post-pool head (reference gnn.py:252-258 with MultiLayerPerceptron / LinearBlock,
 * layers.py:170-267):
 *   y0 = x0 Wp^T + bp
 *   per block i < nb: v_i = y_i W1_i^T + b1_i ; h_i = dropout(act(v_i)) ;
 *                     z_i = h_i W2_i^T + b2_i (+ y_i when skip[i]) ; y_{i+1} = z_i
 *   s = z Ws^T + bs ; cat = [z | s] ; out = cat Wo^T + bo          (z = z_{nb-1})
 * G rows (molecules), F = ffn width (32 <= F <= 256, F % 32 == 0), H_in = input width (% 32 == 0),
 * T outputs. Weights row-major [out, in] (nn.Linear), 16-byte aligned. Dropout: hash mask of
 * (seed, salt 0x4EAD + i, row * F + col), p = drop_p, active when training != 0 and seed != NULL.
 * The forward saves (caller-owned, [G, F] row-major unless noted): y0, v[i], hid[i] (= h_i),
 * mask[i] (uint8, when dropout is active), z[i], cat [G, 2F]; it writes out [G, T] (ld ldo).
 * The backward (AimxHeadGrad) runs the input-gradient chain given d_out: it writes d_x0 and the
 * activation gradients the weight gradients need: ds (= d s), dz[i] (= d z_i), dv[i] (= d v_i),
 * dy0 (= d y0). The weight gradients are then plain dW = dY^T X products (aimx_wgrad_grouped):
 *   Wo: (d_out, cat)  Ws: (ds, z)  W2_i: (dz[i], hid[i])  W1_i: (dv[i], y_i = i ? z[i-1] : y0)
 *   Wp: (dy0, x0)
 * ------------------------------------------------------------------------------------------ */
#define AIMX_HEAD_MAX_BLOCKS 8
#define AIMX_HEAD_SYNC_WORDS 68
typedef struct AimxHead {
  int64_t G, F, H_in, T;
  int32_t nb, act, training;
  float drop_p; const int64_t* seed;
  const float* x0; int64_t ldx0;
  const float* wp; const float* bp;
  const float* w1[AIMX_HEAD_MAX_BLOCKS]; const float* b1[AIMX_HEAD_MAX_BLOCKS];
  const float* w2[AIMX_HEAD_MAX_BLOCKS]; const float* b2[AIMX_HEAD_MAX_BLOCKS];
  int32_t skip[AIMX_HEAD_MAX_BLOCKS];
  const float* ws; const float* bs; const float* wo; const float* bo;
  float* y0; float* v[AIMX_HEAD_MAX_BLOCKS]; float* hid[AIMX_HEAD_MAX_BLOCKS];
  uint8_t* mask[AIMX_HEAD_MAX_BLOCKS]; float* z[AIMX_HEAD_MAX_BLOCKS]; float* cat;
  float* out; int64_t ldo;
  /* Clustered launch: `cluster` (0/1 = off, 2, 4 or 8) workgroups share each 16-molecule tile and
   * exchange activations through HBM inside the launch; `sync` = AIMX_HEAD_SYNC_WORDS int32
   * words, zeroed once by the caller and kept zero by the kernels (word 0 becomes non-zero if a
   * cluster wait ever timed out: results of that call are invalid). */
  int32_t* sync; int32_t cluster;
  /* Forward workspace (aimx_head_forward_workspace_bytes(h), 16-B aligned; NULL: the 16-molecule
   * kernels): the 8-molecule kernels read the transposed chain weights from it. */
  float* fwd_ws; size_t fwd_ws_bytes;
} AimxHead;

typedef struct AimxHeadGrad {
  const float* d_out; int64_t ld_dout;
  float* d_x0; int64_t ld_dx0;
  float* ds; float* dz[AIMX_HEAD_MAX_BLOCKS]; float* dv[AIMX_HEAD_MAX_BLOCKS]; float* dy0;
  void* workspace; size_t workspace_bytes;  /* aimx_head_backward_workspace_bytes(h), 16-B aligned */
} AimxHeadGrad;

size_t aimx_head_forward_workspace_bytes(const AimxHead* h);
int aimx_head_forward(const AimxHead* h, aimx_stream_t stream);
size_t aimx_head_backward_workspace_bytes(const AimxHead* h);
int aimx_head_backward(const AimxHead* h, const AimxHeadGrad* d, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * L1 losses of the train step (reference trainer.py:24-35: nn.L1Loss for one task,
 * WeightedL1Loss src/models/losses.py:14-48 for multitask):
 *   loss = (1/div) * sum_{i<rows, t<cols} w_t |pred[i,t] - target[i,t]|
 *   div = rows (per_sample != 0: sum over tasks, mean over samples) or rows*cols (mean);
 *   weights NULL = all ones. loss is one device float. Backward:
 *   d_pred[i,t] = sign(pred - target) * w_t * d_loss[0] / div  (sign(0) = 0).
 * One deterministic workgroup for the forward (rows*cols is per molecule: a few thousand).
 * ------------------------------------------------------------------------------------------ */
int aimx_l1_loss_forward(const float* pred, int64_t ldp, const float* target, int64_t ldt, int64_t rows,
                         int64_t cols, const float* weights, int32_t per_sample, float* loss,
                         aimx_stream_t stream);
/* The same forward plus the train step's per-step bookkeeping (reference trainer.py:160-171:
 * `torch.isnan(outputs).any()` and `loss.item() * batch_size`, kept on the device so the loop never
 * synchronises), in the loss's own launch:
 *   *loss_sum += loss * scale (fp32 multiply, then fp32 add), *nan_count += any(isnan(pred[:rows])),
 *   *steps += 1.  accum NULL: aimx_l1_loss_forward.
 * d_pred non-NULL: the same launch also writes the backward's d_pred (ld ldd, rows_total rows:
 * rows >= `rows` get 0) for the upstream gradient *d_loss, exactly as
 * aimx_l1_loss_backward_padded would — for a caller that will run the backward with that very
 * d_loss tensor (the captured train step's resident 1), so the backward needs no launch. */
typedef struct AimxLossAccum {
  float* loss_sum;
  int32_t* nan_count;
  int64_t* steps;
  float scale;
  const float* d_loss;
  float* d_pred;
  int64_t ldd;
  int64_t rows_total;
} AimxLossAccum;
int aimx_l1_loss_forward_accum(const float* pred, int64_t ldp, const float* target, int64_t ldt, int64_t rows,
                               int64_t cols, const float* weights, int32_t per_sample, float* loss,
                               const AimxLossAccum* accum, aimx_stream_t stream);
int aimx_l1_loss_backward(const float* pred, int64_t ldp, const float* target, int64_t ldt, int64_t rows,
                          int64_t cols, const float* weights, int32_t per_sample, const float* d_loss,
                          float* d_pred, int64_t ldd, aimx_stream_t stream);
/* The loss over the first `rows` rows of a [rows_total, cols] prediction (the padded static batch
 * of a captured train step: rows >= rows are padding molecules excluded from the loss): d_pred
 * gets the gradient of those rows and 0 for the rest, in one launch (what autograd's
 * slice-backward would otherwise do with a zero fill and a copy). */
int aimx_l1_loss_backward_padded(const float* pred, int64_t ldp, const float* target, int64_t ldt, int64_t rows,
                                 int64_t rows_total, int64_t cols, const float* weights, int32_t per_sample,
                                 const float* d_loss, float* d_pred, int64_t ldd, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Multi-tensor copy: dst_i[0:n_i) = src_i[0:n_i) for every item, in ONE launch per 64 items
 * (src NULL: dst_i filled with zeros). The data-parallel gradient sync packs every bucket's
 * gradients into its flat all-reduce buffer and writes the averaged values back with it
 * (replaces torch.cat + torch._foreach_copy_: measured 8 + 2 x 35 us per c2 step).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  const float* src;
  float* dst;
  int64_t n;
} AimxCopyItem;
int aimx_multi_copy(const AimxCopyItem* items, int32_t n_items, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Stereochemistry features (reference GNN._apply_stereochemistry, gnn.py:310-326, with
 * _cis_trans_calculation gnn.py:452-497 and _tetrahedral_feature_calculation_physics_inspired
 * gnn.py:376-450): out [N, 3D] = [x | ct | tet], the input of stereochemical_embedding_2.
 *   ct  = x + scatter of (-x[cis[0, i]] at cis[1, i]) then (+x[trans[0, i]] at trans[1, i]), i = 0, 1
 *         (rows 0 and 1 of the collated [rows, 2] cis / trans tensors, as the reference indexes
 *         them; rows 0 or >= 2 required, out-of-range atoms skipped)
 *   tet = rows named by a centre: x + the chirality terms of every centre naming them, in item
 *         order; other rows 0; M == 0: tet = x.
 * Tetrahedral items are ordered by a stable CSR of tet.flat (t_rowptr [N+1], t_col [4M]: item ids,
 * aimx_csr_build with key = tet, n_rows = N), so results are deterministic. scratch [4M, D] and
 * stats [M, 8] (floats) are written by the forward and read by the backward; the backward's
 * grad_scratch is another [4M, D]. D <= 1024. All pointers are device memory.
 * ------------------------------------------------------------------------------------------ */
typedef struct AimxStereo {
  const float* x; int64_t ldx, N, D;
  const int64_t* tet; int64_t tet_stride0, tet_stride1, M;
  const int64_t* cis; int64_t cis_stride0, cis_stride1, n_cis;
  const int64_t* trans; int64_t trans_stride0, trans_stride1, n_trans;
  const int32_t* t_rowptr; const int32_t* t_col;
  float* scratch; float* stats;
  float* out; int64_t ldo;
} AimxStereo;
int aimx_stereo_forward(const AimxStereo* p, aimx_stream_t stream);
int aimx_stereo_backward(const AimxStereo* p, const float* d_out, int64_t ld_dout, float* dx, int64_t lddx,
                         float* grad_scratch, aimx_stream_t stream);

/* Dropout seeds of one forward: seeds[0..n) in [0, 2^62) from the device-resident counter state[0]
 * (a splitmix64 sequence), which advances. Replaces the per-forward torch.randint draw, whose
 * CUDA-graph capture adds two generator-state fill launches to every replay; the model seeds the
 * state once from torch's generator, so torch.manual_seed still fixes the masks. */
int aimx_dropout_seeds(int64_t* state, int64_t* seeds, int32_t n, aimx_stream_t stream);

/* Static padded inputs of one shape bucket of the drop-in autograph (aimx/autograph.py): the
 * reference's collated tensors (molecular.py:339-458: 4 int64 feature columns [N], edges [E, 2]
 * int64 (target, source), batch [N] int64, total_charges [G] f32; any element strides) copied
 * into static buffers of Np > N atoms and Ep >= E edges. The Np - N slack atoms form pad_mols
 * padding molecules (ids G .. G + pad_mols - 1, near-equal sizes) and the slack edges are
 * self-pairs over them, so no real molecule's values change (aimx.data.pad_collated's layout).
 * out_feat holds the 4 columns back to back ([4][Np]); out_edges is [Ep, 2] contiguous; one
 * launch. Replaces the per-shape re-collate the reference would need to replay a graph. */
typedef struct AimxPadBatch {
  const int64_t* feat[4];
  int64_t feat_stride[4];
  const int64_t* edges;
  int64_t edge_s0, edge_s1;
  const int64_t* batch;
  int64_t batch_stride;
  const float* charges;
  int64_t charge_stride;
  int64_t N, E, G;
  int64_t* out_feat;
  int64_t* out_edges;
  int64_t* out_batch;
  float* out_charges;
  int64_t Np, Ep, pad_mols;
} AimxPadBatch;
int aimx_pad_batch(const AimxPadBatch* p, aimx_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Gradient all-reduce over RCCL (xGMI inside an MI355X node) — the DDP reducer's collective
 * (reference runner.py:703-707 wraps the model in DistributedDataParallel over "nccl" = RCCL).
 * RCCL is resolved at run time (aimx_comm_load: dlopen of the RCCL the process already uses, e.g.
 * PyTorch's bundled librccl.so, so there is one RCCL instance per process) instead of being a
 * link dependency. A communicator from aimx_comm_init is independent of torch.distributed's, so
 * its collectives can be recorded into a HIP graph (stream capture) without torch's watchdog ever
 * querying their events. aimx_comm_allreduce enqueues ONE ncclAllReduce (fp32, in place) on
 * `stream`: op 0 = sum, 1 = average (ncclAvg: sum / nranks in the same kernel, DDP's averaging).
 * Host-side calls (no device work) except aimx_comm_allreduce.
 * ------------------------------------------------------------------------------------------ */
#define AIMX_COMM_ID_BYTES 128
int aimx_comm_load(const char* rccl_path);
int aimx_comm_unique_id(void* id_out, size_t bytes);
int aimx_comm_init(void** comm_out, const void* id, size_t bytes, int32_t nranks, int32_t rank);
int aimx_comm_allreduce(void* comm, float* buf, int64_t count, int32_t op, aimx_stream_t stream);
int aimx_comm_destroy(void* comm);
/* The bound RCCL's version (ncclGetVersion: major*10000 + minor*100 + patch) and a communicator's
 * rank count (ncclCommCount): the bench line reports what the transport itself says. */
int aimx_comm_version(int32_t* version_out);
int aimx_comm_count(void* comm, int32_t* nranks_out);

#ifdef __cplusplus
}
#endif
#endif /* AIMX_H_ */
