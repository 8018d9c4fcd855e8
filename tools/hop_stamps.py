"""Phase shares of hop_rows.hip's window workgroups from the diagnostic stamp build.

usage: AIMX_LIB_PATH=aimnet-x2d_amd/lib_stamps/libaimx.so python tools/hop_stamps.py [--config c4]
(tools/hop_stamps.sh builds that library with -DAIMX_HOPR_STAMPS). Prints, per window workgroup
and per item, the shader-clock cycles of: scan, peek+issue, sum, barrier after the sum, next-item
LDS writes, store+barrier, settle, and the workgroup's whole life. The stamps' waits change the
timing: read shares, not absolute speed.
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

import bench  # noqa: E402
from aimx import _lib, ops  # noqa: E402
from aimx.plan import GraphPlan  # noqa: E402

NAMES = ["scan_peek", "piece_load", "restage", "bar_restage", "item", "bar_item", "unused"]


def read(lib, reset):
    buf = (ctypes.c_ulonglong * 16)()
    assert lib.aimx_hopr_stamps(buf, 1 if reset else 0) == 0
    return list(buf)


def report(tag, v):
    wgs, items = max(v[9], 1), max(v[7], 1)
    rec = {"case": tag, "window_wgs": v[9], "items": v[7], "life_per_wg": round(v[8] / wgs),
           "per_wg": {n: round(v[i] / wgs) for i, n in enumerate(NAMES)},
           "per_item": {n: round(v[i] / items) for i, n in enumerate(NAMES) if n not in ("scan_peek", "piece_load", "unused")}}
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--atoms", type=int, default=4_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    lib.aimx_hopr_stamps.restype = ctypes.c_int
    lib.aimx_hopr_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    cfg = bench.CONFIGS[a.config]
    batch = bench.make_batches(cfg, 1, 99, dev)[0]
    d, hops = int(0.3 * cfg["hidden"]), cfg["hops"]
    cases = [("in_step", batch.num_atoms)] + ([("roofline", a.atoms)] if a.atoms > 0 else [])
    for label, atoms in cases:
        n0 = batch.num_atoms
        reps = max(1, min(atoms, int(0.95 * (2 ** 31 - 1) / (hops * d))) // n0)
        off = (torch.arange(reps, device=dev, dtype=torch.int64) * n0).view(reps, 1, 1)
        edges = (batch.edges.unsqueeze(0) + off).reshape(-1, 2)
        mol = (batch.batch.unsqueeze(0) + torch.arange(reps, device=dev, dtype=torch.int64).view(reps, 1)
               * batch.num_graphs).reshape(-1)
        n = n0 * reps
        plan = GraphPlan(n, hops, edges=edges, batch=mol, num_graphs=batch.num_graphs * reps)
        x = torch.randn(n, d, device=dev, requires_grad=True)
        for _ in range(2):
            ops.hop(plan, x)
        torch.cuda.synchronize()
        read(lib, True)
        out = ops.hop(plan, x)
        torch.cuda.synchronize()
        report(f"{a.config} {label} fwd ({n} atoms)", read(lib, True))
        out.backward(torch.ones_like(out))
        torch.cuda.synchronize()
        report(f"{a.config} {label} bwd ({n} atoms)", read(lib, True))
        del plan, x, out, edges, mol
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
