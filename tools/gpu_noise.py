"""Diagnose parity noise: error vs fp64 of (a) the reference fp32 (fixture), (b) the oracle's plain
PyTorch ops run in fp32 ON THE GPU (hipBLASLt GEMMs), (c) the HIP path, per tensor."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "aimnet-x2d_amd")]
from golden_cases import load_case  # noqa: E402
from oracle import model as om  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from tools_parity_common import err  # noqa: E402


def oracle_dev(z, cfg, dev, dtype):
    af, edges, batch, tc = load_case_dev(z, dev)
    p = {k: v.to(dev, dtype).requires_grad_() for k, v in om.seeded_params(cfg, int(z["seed"])).items()}
    cap = {}
    out, attn, q = om.gnn_forward(p, cfg, af, edges, batch, tc.to(dtype), capture=cap)
    cap["pre_pool"].retain_grad()
    (out * torch.from_numpy(z["loss_w"]).to(dev, dtype)).sum().backward()
    res = {"out": out, "attn": attn, "pre_pool": cap["pre_pool"], "d_pre_pool": cap["pre_pool"].grad}
    res.update({"grad." + k: v.grad for k, v in p.items() if v.grad is not None})
    return {k: v.detach().double().cpu().numpy() for k, v in res.items() if v is not None}


def load_case_dev(z, dev):
    from golden_cases import case_inputs
    return case_inputs(z, dev)


for name in sys.argv[1:] or ["c5s", "c2"]:
    z, cfg, _ = load_case(name)
    r64 = oracle_dev(z, cfg, "cpu", torch.float64)
    g32 = oracle_dev(z, cfg, "cuda", torch.float32)
    c32 = oracle_dev(z, cfg, "cpu", torch.float32)
    keys = ["out", "attn", "pre_pool", "d_pre_pool"] + [k for k in r64 if "pooling" in k or "embedding_projection" in k]
    print(f"== {name}: tensor  cpu32  gpu-torch32 (vs fp64)")
    for k in keys:
        print(f"   {k:45s} {err(c32[k], r64[k]):.2e}  {err(g32[k], r64[k]):.2e}")


def ours_dev(z, cfg):
    model = T._build_model(cfg, int(z["seed"]))
    cap = {}

    def hook(m, a, o):
        o.retain_grad()
        cap["pre_pool"] = o
    model.concat_self_other.register_forward_hook(hook)
    af, edges, batch, tc = load_case_dev(z, "cuda")
    e0 = torch.empty(0, 2, dtype=torch.long, device="cuda")
    out, attn, q = model(af, edges, batch, tc, torch.empty(0, 4, dtype=torch.long, device="cuda"), e0, e0)
    (out * torch.from_numpy(z["loss_w"]).cuda()).sum().backward()
    res = {"out": out, "attn": attn, "pre_pool": cap["pre_pool"], "d_pre_pool": cap["pre_pool"].grad}
    res.update({"grad." + k: p.grad for k, p in model.named_parameters() if p.grad is not None})
    return {k: v.detach().double().cpu().numpy() for k, v in res.items() if v is not None}


print("== ours (HIP path) vs fp64 on the same tensors")
for name in sys.argv[1:] or ["c5s", "c2"]:
    z, cfg, _ = load_case(name)
    r64 = oracle_dev(z, cfg, "cpu", torch.float64)
    o = ours_dev(z, cfg)
    keys = ["out", "attn", "pre_pool", "d_pre_pool"] + [k for k in r64 if "pooling.attention_weights" in k and "weight" in k] + ["grad.pooling.temperature"]
    print(f"== {name}")
    for k in keys:
        print(f"   {k:45s} {err(o[k], r64[k]):.2e}")
