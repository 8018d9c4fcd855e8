"""Device time of the c2 train step's sections, each captured as its own HIP graph (no profiler):
forward(+loss), forward+backward, and the full step with clip+Adam. Differences give the backward
and optimizer shares without the per-kernel inflation a kernel trace adds.

usage: python tools/step_sections.py [--config c2] [--reps 20] [--env "A=1 B=2" ...]
With --env, the whole-step graph is also captured under each environment setting (AIMX_* knobs
are read at launch/capture time) and all variants are replayed interleaved, so an A/B between
code paths runs on one box in one process.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--env", action="append", default=[])
    a = ap.parse_args()
    from aimx.optim import FusedAdam
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[a.config]
    batches = bench.make_batches(cfg, 2, 1234, dev, pad=True)
    model = bench.build_model(cfg, dev)
    B = cfg["batch"]
    from models import L1Loss
    from aimx import ops
    loss_fn = L1Loss()
    opt = FusedAdam(model.parameters(), lr=2.5e-4, max_grad_norm=1.0)
    static = batches[0].clone()
    one = torch.ones((), dtype=torch.float32, device=dev)

    def fwd():
        out, _, _ = model(*static.model_args())
        return ops.l1_loss(out, static.targets[:B], rows=B)

    sections = {
        "forward+loss": lambda: fwd(),
        "forward+backward": lambda: fwd().backward(one),
        "full step": lambda: (fwd().backward(one), opt.step()),
    }
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            fwd().backward(one)
            opt.step()
    torch.cuda.current_stream().wait_stream(side)
    res = {}
    for name, fn in sections.items():
        opt.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.reps):
            g.replay()
        t1.record()
        t1.synchronize()
        res[name] = round(t0.elapsed_time(t1) / a.reps * 1e3, 1)
        del g
    res["backward"] = round(res["forward+backward"] - res["forward+loss"], 1)
    res["clip+adam"] = round(res["full step"] - res["forward+backward"], 1)
    print(json.dumps({"unit": "us", **res}), flush=True)
    if a.env:
        variants = [""] + a.env
        graphs = []
        for ev in variants:
            kv = [x.split("=") for x in ev.split()]
            for k, v in kv:
                os.environ[k] = v
            with torch.cuda.stream(side):
                opt.zero_grad(set_to_none=True)
                fwd().backward(one)
                opt.step()
            torch.cuda.current_stream().wait_stream(side)
            opt.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fwd().backward(one)
                opt.step()
            for k, _ in kv:
                os.environ.pop(k, None)
            graphs.append(g)
        tot = [0.0] * len(graphs)
        for rnd in range(5):
            for gi, g in enumerate(graphs):
                g.replay()
                torch.cuda.synchronize()
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                for _ in range(a.reps):
                    g.replay()
                t1.record()
                t1.synchronize()
                tot[gi] += t0.elapsed_time(t1) / a.reps * 1e3 / 5
        print(json.dumps({"unit": "us", "ab_full_step": {v or "baseline": round(t, 1) for v, t in zip(variants, tot)}}),
              flush=True)


if __name__ == "__main__":
    main()
