"""Per-tensor parity report of the GPU model against the reference (GPU box).

For every golden case (tests/golden_cases.CASES) and every tensor the case checks (outputs,
attention, partial charges, every parameter gradient, gradient sketches), records:
  vs_ref32  — ours vs the REFERENCE's own fp32 result stored in the fixture (null if not stored)
  vs_fp64   — ours vs the fp64 oracle (the exact answer up to fp64 rounding)
  ref_floor — the reference's own fp32 error vs fp64 (null if not stored)
  tol       — the bound tests/conftest.parity_failures applies: max(1e-5, 3 x ref_floor)
  relaxed   — True where tol > 1e-5, i.e. where the reference itself is further than 1e-5 from
              the exact answer and the 3x-floor rule (not the bare 1e-5) judged the tensor
All errors are norm-relative (max |a - b| / max |b|; attention-bias gradients, exactly 0 in exact
arithmetic, against their weight's scale).

Config-sized cases (c4, c5: test_gpu_parity.FULL_SIZE) carry the oracle's own fp32 run as
`vs_ref32` / `ref_floor` (no reference fixture at that size).

Usage (GPU box): python tools/parity_report.py [--out profiles/r04_parity.json] [case ...]
(default: every golden case, then c4 and c5 at their configured batch)
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "aimnet-x2d_amd")]
from conftest import _scale_for, add_sketches, fixture_refs  # noqa: E402
from golden_cases import CASES, case_stereo, load_case  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def err(a, b, sc):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    den = max(np.abs(b).max() if b.size else 0, sc)
    return float(np.abs(a - b).max() / den) if den > 0 and b.size else 0.0


def run_full(name):
    """A config-sized case (test_gpu_parity.FULL_SIZE: c4 512 x 40-atom molecules, c5 256): the
    reference fp32 floor is the oracle's own fp32 run (the fixture-pinned restatement of the
    reference's ATen ops), every gradient compared whole."""
    z, cfg, inputs, loss_w = T.full_size_case(name)
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    seed = int(z["seed"])
    ref64 = T._run_full(cfg, seed, inputs, loss_w, "cpu", torch.float64)
    ref32 = T._run_full(cfg, seed, inputs, loss_w, "cpu", torch.float32)
    ours = T._run_full(cfg, seed, inputs, loss_w, "cuda")
    return _rows(ours, ref32, ref64)


def run_case(name):
    if name in T.FULL_SIZE:
        return run_full(name)
    z, cfg, inputs = load_case(name)
    torch.set_num_threads(8)
    ref64 = T._oracle_run(z, cfg, inputs, torch.float64)
    ref32 = fixture_refs(z)
    model = T._build_model(cfg, int(z["seed"]))
    af, edges, batch, tc = load_case(name, "cuda")[2]
    out, attn, q = model(af, edges, batch, tc, *case_stereo(z, "cuda"))
    (out * torch.from_numpy(z["loss_w"]).cuda()).sum().backward()
    ours = {"out": out.detach().cpu().numpy()}
    if attn is not None:
        ours["attn"] = attn.detach().cpu().numpy()
    if q is not None:
        ours["q"] = q.detach().cpu().numpy()
    for k, p in model.named_parameters():
        if p.grad is not None:
            ours["grad." + k] = p.grad.cpu().numpy()
    add_sketches(ours, z)
    return _rows(ours, ref32, ref64)


def _rows(ours, ref32, ref64):
    rows = {}
    for k in sorted(ref64):
        if k not in ours:
            continue
        sc = _scale_for(k, ref64)
        e64 = err(ours[k], ref64[k], sc)
        e32 = err(ours[k], ref32[k], sc) if k in ref32 else None
        floor = err(ref32[k], ref64[k], sc) if k in ref32 else None
        tol = max(1e-5, 3.0 * floor) if floor is not None else 1e-5
        rows[k] = {"vs_ref32": e32, "vs_fp64": e64, "ref_floor": floor, "tol": tol, "relaxed": tol > 1e-5,
                   "pass": e64 <= tol}
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("cases", nargs="*")
    a = ap.parse_args()
    report = {"metric": "norm-relative error per tensor (see tools/parity_report.py)", "contract": 1e-5,
              "cases": {}}
    for name in a.cases or (CASES + sorted(T.FULL_SIZE)):
        rows = run_case(name)
        stored = [r for r in rows.values() if r["vs_ref32"] is not None]
        report["cases"][name] = {
            "tensors": len(rows), "vs_ref32_stored": len(stored),
            "max_vs_ref32": max((r["vs_ref32"] for r in stored), default=None),
            "max_vs_fp64": max(r["vs_fp64"] for r in rows.values()),
            "relaxed": sorted(k for k, r in rows.items() if r["relaxed"]),
            "all_pass": all(r["pass"] for r in rows.values()),
            # the literal contract: the fraction of tensors within 1e-5 of fp64, and how close the
            # rest come to the bound they are judged by (error / the reference's own fp32 floor)
            "frac_within_1e-5": sum(r["vs_fp64"] <= 1e-5 for r in rows.values()) / max(len(rows), 1),
            "max_err_over_floor": max((r["vs_fp64"] / r["ref_floor"] for r in rows.values()
                                       if r["ref_floor"]), default=None),
            "max_err_over_tol": max(r["vs_fp64"] / r["tol"] for r in rows.values()),
            "per_tensor": rows,
        }
        c = report["cases"][name]
        print(f"{name:12s} tensors {c['tensors']:3d}  max vs fp64 {c['max_vs_fp64']:.2e}  within 1e-5 "
              f"{c['frac_within_1e-5']:.2f}  max err/tol {c['max_err_over_tol']:.2f}  relaxed {c['relaxed']}  "
              f"pass {c['all_pass']}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
