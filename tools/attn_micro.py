"""Attention-pool kernels at the bench configs' sizes: forward and backward launch time (HIP events
around 50 back-to-back launches; run under rocprofv3 --kernel-trace for per-kernel durations), achieved GB/s on the algorithmic bytes, fraction of
8 TB/s.

Algorithmic bytes per launch (fp32):
  fwd = 4 * (N*C  [read x] + 2*H*N [write attn, scores] + G*C [write pooled] + H*C [read W])
  bwd = 4 * (2*N*C [read x, write dx] + 2*H*N [read attn, scores] + G*C [read dpooled] + H*C [read W, write dW])

Usage: python tools/attn_micro.py [--json OUT]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

# (name, molecules, mean atoms, hidden, heads): c2/c3 QM9-shaped, c4 40-atom h512, c5 40-atom h1024
CONFIGS = [("c2", 512, 18, 256, 4), ("c4", 512, 40, 512, 4), ("c5", 256, 40, 1024, 4)]


def timed(fn, it=50):
    """Mean launch time over `it` back-to-back launches on the current stream (HIP events)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(it):
        fn()
    t1.record()
    t1.synchronize()
    return t0.elapsed_time(t1) / it * 1e3  # us per launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    a = ap.parse_args()
    import aimx
    from aimx import _lib
    from aimx.plan import GraphPlan  # noqa: F401
    from models.pooling import MultiHeadAttentionPoolingLayer, _plan_for
    lib = aimx.load()
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    out = []
    for name, G, mean_atoms, C, H in CONFIGS:
        sizes = np.clip(rng.normal(mean_atoms, 2 if mean_atoms > 20 else 3, G).round().astype(int), 3, 60)
        batch = torch.from_numpy(np.repeat(np.arange(G), sizes)).to(dev)
        N = int(sizes.sum())
        x = torch.randn(N, C, device=dev)
        pool = MultiHeadAttentionPoolingLayer(C, num_heads=H).to(dev)
        plan = _plan_for(pool, x, batch)
        W = torch.cat([lin.weight for lin in pool.attention_weights], 0).contiguous()
        b = torch.cat([lin.bias for lin in pool.attention_weights], 0).contiguous()
        tau = pool.temperature.detach().float().contiguous()
        pooled = torch.empty(G, C, device=dev)
        attn = torch.empty(H, N, device=dev)
        scores = torch.empty(H, N, device=dev)
        dpool = torch.randn(G, C, device=dev)
        dx = torch.empty(N, C, device=dev)
        dW = torch.empty(H, C, device=dev)
        db = torch.empty(H, device=dev)
        dtau = torch.empty(1, device=dev)
        wsb = lib.aimx_attn_pool_workspace_bytes(N, C, H, G)
        ws = torch.empty(wsb // 4 + 1, device=dev)
        P = _lib.ptr
        rp, col = P(plan.graph.rowptr), P(plan.graph.col)

        def fwd():
            s = _lib.stream_ptr(dev)
            assert lib.aimx_attn_pool_forward(P(x), C, N, C, P(W), P(b), P(tau), H, rp, col, G, P(pooled), P(attn),
                                              P(scores), s) == 0

        def bwd():
            s = _lib.stream_ptr(dev)
            assert lib.aimx_attn_pool_backward(P(x), C, N, C, P(W), P(tau), H, rp, col, G, P(attn), P(scores),
                                               P(dpool), None, P(dx), C, P(dW), P(db), P(dtau), P(ws), wsb, s) == 0

        tf, tb = timed(fwd), timed(bwd)
        bf = 4 * (N * C + 2 * H * N + G * C + H * C)
        bb = 4 * (2 * N * C + 2 * H * N + G * C + 2 * H * C)
        r = {"config": name, "G": G, "N": N, "C": C, "H": H, "fwd_us": round(tf, 2), "bwd_us": round(tb, 2),
             "fwd_bytes": bf, "bwd_bytes": bb, "fwd_GBps": round(bf / tf / 1e3, 1), "bwd_GBps": round(bb / tb / 1e3, 1),
             "fwd_frac": round(bf / tf / 1e3 / 8000, 4), "bwd_frac": round(bb / tb / 1e3 / 8000, 4)}
        print(json.dumps(r), flush=True)
        out.append(r)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
