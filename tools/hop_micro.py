"""Hop kernel micro-benchmark at roofline size: separates the gather phase (chunk 0) from the
zero-store phase (chunks 1..h-1) and prints copy / fill reference rates on the same device.

usage: python tools/hop_micro.py [--atoms 4000000] [--launches 20] [--env "A=1 B=2" ...] [--rounds 2]
Each line: {"case", "ms", "alg_GBs"} (algorithmic bytes of that case / time). With --env, the hop
cases run once per environment setting, each in a child process (the launcher reads its AIMX_HOP_*
knobs once per process), interleaved over --rounds rounds so that drift cancels in the comparison.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

import bench  # noqa: E402
from aimx import ops  # noqa: E402
from aimx.plan import GraphPlan  # noqa: E402


def timeit(fn, launches):
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(s)
    for _ in range(launches):
        fn()
    t1.record(s)
    t1.synchronize()
    return t0.elapsed_time(t1) / launches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--atoms", type=int, default=4_000_000)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    if a.env:
        import subprocess
        for rnd in range(a.rounds):
            for ev in a.env:
                env = dict(os.environ)
                for kv in ev.replace(",", " ").split():
                    k, v = kv.split("=")
                    env[k] = v
                subprocess.run([sys.executable, os.path.abspath(__file__), "--atoms", str(a.atoms), "--launches",
                                str(a.launches), "--label", f"[{ev}] r{rnd}"], env=env, check=True)
        return
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS["c2"]
    batch = bench.make_batches(cfg, 1, 99, dev)[0]
    n0, d = batch.num_atoms, int(0.3 * cfg["hidden"])
    reps = max(1, a.atoms // n0)
    off = (torch.arange(reps, device=dev, dtype=torch.int64) * n0).view(reps, 1, 1)
    edges = (batch.edges.unsqueeze(0) + off).reshape(-1, 2)
    n, e = n0 * reps, edges.shape[0]
    x = torch.randn(n, d, device=dev)
    out = []
    g0 = batch.num_graphs
    mol = (batch.batch.unsqueeze(0) + torch.arange(reps, device=dev, dtype=torch.int64).view(reps, 1) * g0).reshape(-1)
    plans = {h: GraphPlan(n, h, edges=edges, batch=mol, num_graphs=g0 * reps) for h in (3, 1)}
    for rnd in range(a.rounds):
        for h in (3, 1):
            plan = plans[h]
            ms = timeit(lambda: ops.hop(plan, x), a.launches)
            b = 4 * (n * d + e + (h * n + 1) + h * n * d)
            out.append({"case": f"hop h={h} {a.label} r{rnd}", "ms": ms, "alg_GBs": b / ms / 1e6})
            print(json.dumps(out[-1]), flush=True)
    del plans
    plan = GraphPlan(n, 2, edges=edges[:0])
    ms = timeit(lambda: ops.hop(plan, x), a.launches)
    out.append({"case": "hop h=2, E=0 (zero stores)", "ms": ms, "alg_GBs": 4 * (2 * n + 1 + 2 * n * d) / ms / 1e6})
    del plan
    z = torch.empty(2 * n, d, device=dev)
    ms = timeit(lambda: z.zero_(), a.launches)
    out.append({"case": "torch zero_ same bytes", "ms": ms, "alg_GBs": 4 * 2 * n * d / ms / 1e6})
    y = torch.empty_like(x)
    ms = timeit(lambda: y.copy_(x), a.launches)
    out.append({"case": "torch copy_ x", "ms": ms, "alg_GBs": 8 * n * d / ms / 1e6})
    for r in out[-3:]:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
