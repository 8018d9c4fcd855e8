"""A/B of the stack's weight gradients: aimx_wgrad_grouped (k_wgrad_lds) against the vendor GEMM
(torch.mm -> hipBLASLt / rocBLAS, fp32) on the same dW = dY^T X problems, graph-timed.
Problems per layer: dW_ig (2D x (h+1)D, the untrimmed input projection) and 4 x dW_mlp (D x D);
bias columns excluded on the vendor side (a column sum, timed separately).
usage: python tools/wgrad_lib_ab.py [c4|c5] [pad]   (pad: row strides rounded up to 4 floats, 16-byte rows)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
from aimx import _lib  # noqa: E402


def graph_us(fn, reps=10, rounds=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(rounds):
        g.replay()
    t1.record()
    t1.synchronize()
    return t0.elapsed_time(t1) / (reps * rounds) * 1e3


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    K, D, h = {"c4": (20480, 153, 3), "c5": (10240, 307, 6)}[cfg]
    pad = len(sys.argv) > 2 and sys.argv[2] == "pad"
    groups = {"wig": [(2 * D, (h + 1) * D)] * 3, "mlp": [(D, D)] * 12}
    groups["all"] = groups["wig"] + groups["mlp"]
    res = {"config": cfg, "K": K, "D": D, "hops": h, "pad": pad}
    for name, shapes in groups.items():
        flops = sum(2 * M * N * K for M, N in shapes)
        ops, arr = [], (_lib.WgradProblem * len(shapes))()
        for i, (M, N) in enumerate(shapes):
            lm, ln = (-(-M // 4) * 4, -(-N // 4) * 4) if pad else (M, N)
            dy, x = torch.randn(K, lm, device=dev)[:, :M], torch.randn(K, ln, device=dev)[:, :N]
            dw, db = torch.empty(M, N, device=dev), torch.empty(M, device=dev)
            ops.append((dy, x, dw, db))
            arr[i].dY, arr[i].ld_dy, arr[i].X, arr[i].ld_x = dy.data_ptr(), lm, x.data_ptr(), ln
            arr[i].dW, arr[i].ld_dw, arr[i].col_out = dw.data_ptr(), N, db.data_ptr()
            arr[i].M, arr[i].N, arr[i].K = M, N, K
        n = len(shapes)
        ws = torch.empty(lib.aimx_wgrad_grouped_workspace_bytes(arr, n) // 4 + 1, device=dev)
        cnt = _lib.counters(dev)
        ours = lambda: lib.aimx_wgrad_grouped(arr, n, ws.data_ptr(), ws.numel() * 4, cnt.data_ptr(), _lib.N_COUNTERS,
                                              torch.cuda.current_stream().cuda_stream)

        def vendor():
            for dy, x, dw, db in ops:
                torch.mm(dy.t(), x, out=dw)

        def vendor_bias():
            for dy, x, dw, db in ops:
                torch.mm(dy.t(), x, out=dw)
                torch.sum(dy, 0, out=db)

        # the two paths agree (fp32, different summation orders)
        ours()
        torch.cuda.synchronize()
        ref = [dw.clone() for _, _, dw, _ in ops]
        vendor()
        torch.cuda.synchronize()
        err = max(float((r - dw).norm() / dw.norm()) for r, (_, _, dw, _) in zip(ref, ops))
        r = {"gflop": round(flops / 1e9, 2), "rel_diff": err}
        for tag, fn in (("aimx", ours), ("vendor", vendor), ("vendor_bias", vendor_bias)):
            us = graph_us(fn)
            r[tag + "_us"] = round(us, 1)
            r[tag + "_tfs"] = round(flops / us / 1e6, 1)
        res[name] = r
        del ops, ws
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
