"""The hop backward alone at bench.py's roofline size (for rocprofv3 --pmc passes).
usage: python tools/hop_bwd_only.py [--config c5] [--fwd]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

import bench  # noqa: E402
from aimx import ops  # noqa: E402
from aimx.plan import GraphPlan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--fwd", action="store_true")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    batch = bench.make_batches(cfg, 1, 99, dev)[0]
    hops, d = cfg["hops"], int(0.3 * cfg["hidden"])
    n0 = batch.num_atoms
    target = min(4_000_000, int(0.95 * (2 ** 31 - 1) / (hops * d)))
    reps = max(1, target // n0)
    off = (torch.arange(reps, device=dev, dtype=torch.int64) * n0).view(reps, 1, 1)
    edges = (batch.edges.unsqueeze(0) + off).reshape(-1, 2)
    mol = batch.batch.unsqueeze(0) + torch.arange(reps, device=dev, dtype=torch.int64).view(reps, 1) * batch.num_graphs
    plan = GraphPlan(n0 * reps, hops, edges=edges, batch=mol.reshape(-1), num_graphs=batch.num_graphs * reps)
    if a.fwd:
        x = torch.randn(plan.N, d, device=dev)
        for _ in range(5):
            ops.hop(plan, x)
    else:
        r = bench.hop_bwd_roofline(plan, plan.N, d, hops, dev, launches=5)
        print(r)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
