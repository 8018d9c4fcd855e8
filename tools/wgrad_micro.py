"""Graph-timed aimx_wgrad_grouped on a stack's 15 weight-gradient problems (3 layers x
[dW_ig 2D x 2D + bias (the trimmed input projection), 4 x dW_mlp D x D + bias]), K = atoms.
usage: python tools/wgrad_micro.py [c2|c4|c5] [KPER,KPER,...]   (AIMX_WGRAD_KPER sweep)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
from aimx import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    K, D = {"c2": (9170, 76), "c4": (20480, 153), "c5": (10240, 307)}[cfg]
    kpers = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    shapes = [(2 * D, 2 * D)] + [(D, D)] * 4
    shapes = shapes * 3
    flops = sum(2 * M * (N + 1) * K for M, N in shapes)
    bufs = []
    arr = (_lib.WgradProblem * len(shapes))()
    for i, (M, N) in enumerate(shapes):
        # rows rounded to 4 floats, as the stack lays them out (16-byte staging)
        lm, ln = (M + 3) // 4 * 4, (N + 3) // 4 * 4
        dy, x = torch.randn(K, lm, device=dev), torch.randn(K, ln, device=dev)
        dw, db = torch.empty(M, N, device=dev), torch.empty(M, device=dev)
        bufs += [dy, x, dw, db]
        arr[i].dY, arr[i].ld_dy, arr[i].X, arr[i].ld_x = dy.data_ptr(), lm, x.data_ptr(), ln
        arr[i].dW, arr[i].ld_dw, arr[i].col_out = dw.data_ptr(), N, db.data_ptr()
        arr[i].M, arr[i].N, arr[i].K = M, N, K
    n = len(shapes)
    ws = torch.empty(lib.aimx_wgrad_grouped_workspace_bytes(arr, n) // 4 + 1, device=dev)
    cnt = _lib.counters(dev)
    res = {"config": cfg, "K": K, "D": D, "gflop": round(flops / 1e9, 2)}
    for kper in kpers:
        path = f"kper{kper}" if kper else "default"
        if kper:
            os.environ["AIMX_WGRAD_KPER"] = str(kper)
        else:
            os.environ.pop("AIMX_WGRAD_KPER", None)
        ws = torch.empty(lib.aimx_wgrad_grouped_workspace_bytes(arr, n) // 4 + 1, device=dev)
        fn = lambda: lib.aimx_wgrad_grouped(arr, n, ws.data_ptr(), ws.numel() * 4, cnt.data_ptr(), _lib.N_COUNTERS,
                                            torch.cuda.current_stream().cuda_stream)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(10):
                fn()
        g.replay()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(5):
            g.replay()
        t1.record()
        t1.synchronize()
        us = t0.elapsed_time(t1) / 50 * 1e3
        res[path + "_us"] = round(us, 1)
        res[path + "_tfs"] = round(flops / us / 1e6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
