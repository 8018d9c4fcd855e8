"""Per-tensor parity report on the GPU: err(ours vs fp64 oracle) next to err(reference fp32 vs fp64).

Usage (GPU box): python tools/parity_report.py [case ...]  -> prints the worst tensors per case.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "aimnet-x2d_amd")]
from conftest import _scale_for  # noqa: E402
from golden_cases import CASES, load_case  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def err(a, b, sc):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    den = max(np.abs(b).max() if b.size else 0, sc)
    return np.abs(a - b).max() / den if den > 0 else 0.0


def main(cases):
    worst_ratio = []
    for name in cases:
        z, cfg, inputs = load_case(name)
        ref64 = T._oracle_run(z, cfg, inputs, torch.float64)
        model = T._build_model(cfg, int(z["seed"]))
        af, edges, batch, tc = load_case(name, "cuda")[2]
        e0 = torch.empty(0, 2, dtype=torch.long, device="cuda")
        out, attn, q = model(af, edges, batch, tc, torch.empty(0, 4, dtype=torch.long, device="cuda"), e0, e0)
        (out * torch.from_numpy(z["loss_w"]).cuda()).sum().backward()
        ours = {"out": out.detach().cpu().numpy()}
        if attn is not None:
            ours["attn"] = attn.detach().cpu().numpy()
        if q is not None:
            ours["q"] = q.detach().cpu().numpy()
        for k, p in model.named_parameters():
            if p.grad is not None:
                ours["grad." + k] = p.grad.cpu().numpy()
        rows = []
        for k in ref64:
            if k not in ours:
                continue
            sc = _scale_for(k, ref64)
            e_o = err(ours[k], ref64[k], sc)
            e_r = err(z[k], ref64[k], sc) if k in z.files else float("nan")
            rows.append((e_o, e_r, k))
        rows.sort(reverse=True)
        print(f"== {name}: {len(rows)} tensors; worst ours-vs-fp64 (ref32-vs-fp64):")
        for e_o, e_r, k in rows[:6]:
            print(f"   {k:55s} {e_o:.2e}  ({e_r:.2e})")
        worst_ratio.append(max((e_o / max(e_r, 1e-7), k) for e_o, e_r, k in rows if e_r == e_r))
    print("max ours/ref ratios:", [(f"{r:.1f}", k) for r, k in worst_ratio])


if __name__ == "__main__":
    main(sys.argv[1:] or CASES)
