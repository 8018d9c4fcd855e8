"""Per-node cost of a captured HIP graph of trivial kernels (the launch floor in graph replay).

usage: python tools/launch_floor.py [--nodes 200]
Prints ms per replay / nodes for a chain of 1-element torch ops, and for a chain of 1-WG aimx
copy kernels (aimx_copy2d via ctypes if exported), each in its own graph.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=200)
    a = ap.parse_args()
    x = torch.zeros(1, device="cuda")
    big = torch.zeros(1 << 20, device="cuda")
    s = torch.cuda.Stream()
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_CLR", "HIP_", "AMD_"))}}
    for name, fn in (("add_1elem", lambda: x.add_(1.0)), ("add_1M", lambda: big.add_(1.0))):
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(a.nodes):
                fn()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(10):
            g.replay()
        t1.record()
        t1.synchronize()
        res[f"graph_{name}_us_per_node"] = round(t0.elapsed_time(t1) / 10 / a.nodes * 1e3, 3)
        # eager from python (host-bound if the host is slower than the device)
        torch.cuda.synchronize()
        t0.record()
        for _ in range(a.nodes):
            fn()
        t1.record()
        t1.synchronize()
        res[f"eager_{name}_us_per_op"] = round(t0.elapsed_time(t1) / a.nodes * 1e3, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
