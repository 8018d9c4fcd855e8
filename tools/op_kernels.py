"""Which Python-level op launches each GPU kernel of one eager c2 train step (torch.profiler): prints
the kernels in launch order with the innermost CPU op that launched them, so glue launches (fills,
cats, copies) can be traced to their source line.

usage: python tools/op_kernels.py [--config c2]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    a = ap.parse_args()
    import bench
    from aimx.optim import FusedAdam
    from models import L1Loss
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda")
    model = bench.build_model(cfg, dev)
    opt = FusedAdam(model.parameters(), lr=2.5e-4, max_grad_norm=1.0)
    crit = L1Loss()
    b = bench.make_batches(cfg, 1, 5, dev, pad=True)[0]
    B = cfg["batch"]
    ls, nc, st = (torch.zeros((), device=dev), torch.zeros((), dtype=torch.int32, device=dev),
                  torch.zeros((), dtype=torch.int64, device=dev))
    one = torch.ones((), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        out, _, _ = model(*b.model_args())
        loss = crit.padded(out, b.targets[:B], B, accum=(ls, nc, st, float(B)))
        loss.backward(one)
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    evs = sorted(prof.events(), key=lambda e: e.time_range.start)
    for e in evs:
        ks = getattr(e, "kernels", None)
        if not ks:
            continue
        frames = [f for f in (e.stack or []) if "aimnet-x2d_amd" in f or "bench.py" in f or "tools/" in f]
        for k in ks:
            print(f"{k.name[:70]:70s} <- {e.name[:40]:40s} {frames[0][:120] if frames else ''}")


if __name__ == "__main__":
    main()
