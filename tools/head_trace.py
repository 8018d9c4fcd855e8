"""Phase timestamps of the fused head kernels (diagnostics build: make CXXFLAGS+=-DAIMX_HEAD_TRACE).
Runs the c2-shaped head forward+backward for each AIMX_HEAD_CLUSTER[wWAVES] config in HEAD_CLUSTERS
and prints, for workgroup 0 and workgroup grid/2, the microseconds of each phase (GEMM, exchange)."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]


def main():
    from aimx import _lib, ops
    lib = _lib.load()
    lib.aimx_head_trace_read.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    F, G = 256, 520
    mk = lambda *s: (torch.randn(*s, generator=g) * 0.05).to(dev).requires_grad_()  # noqa: E731
    x = mk(G, F)
    wp, bp = mk(F, F), mk(F)
    blocks = [(mk(F, F), mk(F), mk(F, F), mk(F)) for _ in range(3)]
    ws, bs, wo, bo = mk(F, F), mk(F), mk(1, 2 * F), mk(1)
    for cfg in os.environ.get("HEAD_CLUSTERS", "1,4").split(","):
        S, _, W = cfg.partition("w")
        os.environ["AIMX_HEAD_CLUSTER"] = S
        if W:
            os.environ["AIMX_HEAD_WAVES"] = W
        else:
            os.environ.pop("AIMX_HEAD_WAVES", None)
        for _ in range(5):
            y = ops.head(x, wp, bp, blocks, ws, bs, wo, bo, act="silu", drop_p=0.05, training=True,
                         skips=[False, True, True])
            y.sum().backward()
        torch.cuda.synchronize()
        buf = (ctypes.c_longlong * 128)()
        lib.aimx_head_trace_read(ctypes.addressof(buf))
        t = list(buf)
        out = {}
        for wg in range(2):
            row = t[wg * 64:(wg + 1) * 64]
            for part, lo in (("fwd", 0), ("bwd", 32)):
                st = [v for v in row[lo:lo + 32] if v]
                out[f"wg{wg}_{part}"] = [round((b - a) / 100.0, 2) for a, b in zip(st, st[1:])]
                out[f"wg{wg}_{part}_total"] = round((st[-1] - st[0]) / 100.0, 2) if st else None
        print(json.dumps({cfg: out}), flush=True)


if __name__ == "__main__":
    main()
