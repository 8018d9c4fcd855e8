"""Microbenchmark of aimx_gemm vs torch (hipBLASLt) on the hot path's GEMM shapes."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
from aimx import _lib  # noqa: E402

lib = _lib.load()
dev = "cuda"


def bench(fn, it=50):
    """us per launch, measured on a HIP graph of `it` back-to-back launches (device time incl. the
    ~1.6 us graph-node floor; eager Python launches would measure the host instead)."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(5):
        g.replay()
    t1.record()
    t1.synchronize()
    return t0.elapsed_time(t1) / (5 * it) * 1e3


def run(M, N, K, layout, label, splits=0, torch_ref=True, counters=True, lda=None, ldb=None):
    """lda / ldb: row strides of A / B as stored (the step's padded or odd strides; default dense)."""
    if layout[0] == "N":
        A = torch.randn(M, lda or K, device=dev)[:, :K]
    else:
        A = torch.randn(K, lda or M, device=dev)[:, :M]
    if layout[1] == "N":
        B = torch.randn(K, ldb or N, device=dev)[:, :N]
    else:
        B = torch.randn(N, ldb or K, device=dev)[:, :K]
    C = torch.empty(M, N, device=dev)
    a = _lib.GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.A = A.data_ptr()
    a.sam, a.sak = (A.stride(0), 1) if layout[0] == "N" else (1, A.stride(0))
    a.B = B.data_ptr()
    a.sbk, a.sbn = (B.stride(0), 1) if layout[1] == "N" else (1, B.stride(0))
    a.C, a.ldc = C.data_ptr(), N
    a.act, a.dact_kind = -1, -1
    a.splits = splits
    if counters:
        a.counters, a.n_counters = _lib.counters(dev).data_ptr(), _lib.N_COUNTERS
    wsb = lib.aimx_gemm_workspace_bytes(ctypes.byref(a))
    ws = torch.empty(wsb // 4 + 1, device=dev)
    a.workspace, a.workspace_bytes = ws.data_ptr(), wsb
    t_ours = bench(lambda: lib.aimx_gemm(ctypes.byref(a), torch.cuda.current_stream().cuda_stream))
    Am = A if layout[0] == "N" else A.t()
    Bm = B if layout[1] == "N" else B.t()
    t_torch = bench(lambda: torch.mm(Am, Bm, out=C)) if torch_ref else float("nan")
    fl = 2 * M * N * K
    print(f"{label:28s} M={M:6d} N={N:5d} K={K:6d} {layout}: ours {t_ours:7.1f} us ({fl / t_ours / 1e6:6.1f} TF/s)"
          f"  torch {t_torch:7.1f} us ({fl / t_torch / 1e6:6.1f} TF/s)")


if len(sys.argv) > 1 and sys.argv[1] == "big":
    # the c2 / c4 / c5 GEMMs in the step's layouts (hipBLASLt as a yardstick only): embedding
    # projection, [Wi; Wg] input projection (K trimmed to the non-empty chunks, weight rows of the
    # full D(h+1)), its input gradient, the node-update D x D, the concat and its input gradient
    for M, D, h, H in ((9170, 76, 3, 256), (20480, 153, 3, 512), (10240, 307, 6, 1024)):
        K_ig = D * (h + 1)
        run(M, H, 256, "NT", f"h{H} embed proj")
        run(M, 2 * D, 2 * D, "NT", f"h{H} [u|g] fwd (zc)", lda=(K_ig + 3) // 4 * 4, ldb=K_ig)
        run(M, 2 * D, 2 * D, "NN", f"h{H} [u|g] dF (zc)", lda=(2 * D + 3) // 4 * 4, ldb=K_ig)
        run(M, D, D, "NT", f"h{H} node fwd")
        run(M, D, D, "NN", f"h{H} node dX")
        run(M, H, H, "NT", f"h{H} concat fwd")
        run(M, H, H, "NN", f"h{H} concat dX")
        run(H, H + 1, M, "TN", f"h{H} concat dW")
    sys.exit(0)

if len(sys.argv) > 1 and sys.argv[1] == "slices":
    # per-slice latency: one split, few tiles, K swept (no reduction, idle chip)
    for K in (512, 1024, 2048, 4096, 8192):
        run(76, 77, K, "TN", f"dW mlp S=1 K={K}", splits=1, torch_ref=False)
    for K in (512, 1024, 2048, 4096, 8192):
        run(64, 64, K, "NT", f"NT 64x64 S=1 K={K}", splits=1, torch_ref=False)
    sys.exit(0)

if len(sys.argv) > 1 and sys.argv[1] == "dw":
    for M, N, K, lab in [(76, 77, 9170, "c2 dW mlp"), (152, 305, 9170, "c2 dW_ig"), (256, 257, 9170, "c2 concat dW"),
                         (256, 257, 520, "c2 ffn dW")]:
        for sp in (0, 4, 8, 16, 32):
            run(M, N, K, "TN", f"{lab} splits={sp}", splits=sp, torch_ref=False)
    sys.exit(0)

if len(sys.argv) > 1 and sys.argv[1] == "node":
    # the c4 / c5 node-update GEMMs (D = 153 / 307) against the same GEMMs at widths padded to 4 / 16
    for M, D in ((20800, 153), (10240, 307)):
        for w in (D, (D + 3) // 4 * 4, (D + 15) // 16 * 16):
            run(M, w, w, "NT", f"node fwd D={D} w={w}")
            run(M, w, w, "NN", f"node bwd D={D} w={w}")
    sys.exit(0)

if len(sys.argv) > 1 and sys.argv[1] == "head":
    # c5's post-pool chain (F = 1024, 256 molecules + up to 2 padding): forward, input gradient,
    # weight gradient, at the planner's choice and with forced splits
    for M in (256, 258):
        for sp in (0, 1, 2, 4, 8):
            run(M, 1024, 1024, "NT", f"c5 head fwd splits={sp}", splits=sp)
            run(M, 1024, 1024, "NN", f"c5 head dX splits={sp}", splits=sp, torch_ref=sp == 0)
        run(1024, 1024, M, "TN", "c5 head dW")
    sys.exit(0)

if len(sys.argv) > 1 and sys.argv[1] == "deep":
    # k_gemm_deep's shapes: c5's post-pool chain (256 molecules, F = 1024) forward / input gradient,
    # its output layer (K = 2F) and c4's F = 512 chain (AIMX_GEMM_DEEP in the tuning build: 16 / 8 / 0)
    run(256, 1024, 1024, "NT", "c5 head fwd")
    run(256, 1024, 1024, "NN", "c5 head dX")
    run(256, 1, 2048, "NT", "c5 output layer")
    run(256, 2048, 1, "NN", "c5 output dX", torch_ref=False)
    run(512, 512, 512, "NT", "c4 head fwd")
    run(512, 512, 512, "NN", "c4 head dX")
    sys.exit(0)

if len(sys.argv) > 1 and sys.argv[1] == "ugpad":
    # c4 / c5 [Wi; Wg] products with the weight rows at their reference stride D(h+1) (odd: dword
    # staging) against a stride rounded to 4 floats (16-byte staging)
    for M, D, h in ((20480, 153, 3), (10240, 307, 6)):
        K_ig = D * (h + 1)
        ldf = (K_ig + 3) // 4 * 4
        for ldb in (K_ig, ldf):
            run(M, 2 * D, 2 * D, "NT", f"D{D} [u|g] fwd ldb={ldb}", lda=ldf, ldb=ldb, torch_ref=False)
            run(M, 2 * D, 2 * D, "NN", f"D{D} [u|g] dF ldb={ldb}", lda=(2 * D + 3) // 4 * 4, ldb=ldb, torch_ref=False)
    sys.exit(0)

if len(sys.argv) > 1 and sys.argv[1] == "splits":
    for M, N, K, lab in [(76, 77, 9170, "c2 dW mlp"), (152, 305, 9170, "c2 dW_ig"), (256, 257, 9170, "c2 concat dW")]:
        for sp in (0, 4, 8, 12, 16, 24, 32, 48, 64):
            run(M, N, K, "TN", f"{lab} splits={sp}", splits=sp, torch_ref=False)
            run(M, N, K, "TN", f"{lab} splits={sp} 2-kernel", splits=sp, torch_ref=False, counters=False)
    sys.exit(0)

for args in [(9170, 152, 304, "NT", "c2 fwd [u|g]"), (9170, 76, 76, "NT", "c2 fwd mlp"),
             (9170, 304, 152, "NN", "c2 bwd dF"), (9170, 76, 76, "NN", "c2 bwd dx mlp"),
             (152, 305, 9170, "TN", "c2 dW_ig"), (76, 77, 9170, "TN", "c2 dW mlp"),
             (512, 256, 256, "NT", "c2 ffn fwd"), (256, 257, 512, "TN", "c2 ffn dW"),
             (9170, 256, 256, "NT", "c2 concat fwd"), (256, 257, 9170, "TN", "c2 concat dW"),
             (20480, 306, 612, "NT", "c4 fwd [u|g]"), (10240, 614, 2149, "NT", "c5 fwd [u|g]"),
             (4096, 4096, 4096, "NT", "square 4k")]:
    run(*args)
