"""Measure the intrinsic fp32 noise floor of each golden case: oracle fp32 vs oracle fp64.

Prints per-tensor norm-relative errors (max|d|/max|ref|). Used to justify the parity tolerances
stated in tests.
"""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "aimnet-x2d_amd")]
from conftest import norm_rel
from golden_cases import CASES, load_case
from oracle import model as om

def run(name, dtype):
    z, cfg, (af, edges, batch, tc) = load_case(name)
    p = {k: v.to(dtype).requires_grad_() for k, v in om.seeded_params(cfg, int(z["seed"])).items()}
    out, attn, q = om.gnn_forward(p, cfg, af, edges, batch, tc.to(dtype))
    (out * torch.from_numpy(z["loss_w"]).to(dtype)).sum().backward()
    res = {"out": out.detach().double().numpy()}
    if attn is not None: res["attn"] = attn.detach().double().numpy()
    if q is not None: res["q"] = q.detach().double().numpy()
    for k, v in p.items():
        if v.grad is not None: res["grad." + k] = v.grad.double().numpy()
    return z, res

for name in (sys.argv[1:] or CASES):
    z, r32 = run(name, torch.float32)
    _, r64 = run(name, torch.float64)
    worst = sorted(((norm_rel(r32[k], r64[k]), k) for k in r32), reverse=True)[:4]
    ref = {k: norm_rel(z[k], r64[k]) for k in ("out", "attn", "q") if k in z.files}
    print(f"{name:14s} fp32-vs-fp64 out={norm_rel(r32['out'], r64['out']):.2e} worst={[(k, f'{e:.1e}') for e, k in worst]} reference-vs-fp64={ {k: f'{v:.1e}' for k, v in ref.items()} }")
