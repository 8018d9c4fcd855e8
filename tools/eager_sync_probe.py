"""Eager (drop-in) c2 step: does it synchronise with the device, and how long does the host take to
enqueue one step? Prints torch's sync-debug warnings (one per synchronising call site) and the
enqueue-only vs end-to-end ms per step."""
import os
import sys
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bs = bench.make_batches(cfg, 4, 777, dev, pad=False)
    model = bench.build_model(cfg, dev)
    from aimx.optim import FusedAdam
    from models import L1Loss
    loss_fn, opt = L1Loss(), FusedAdam(model.parameters(), lr=2.5e-4, max_grad_norm=1.0)

    def step(i):
        b = bs[i % len(bs)]
        opt.zero_grad(set_to_none=True)
        out, _, _ = model(*b.model_args())
        loss_fn(out, b.targets).backward()
        opt.step()
    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("warn")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        step(0)
        torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode(0)
    seen = set()
    for x in w:
        k = str(x.message)[:200]
        if k not in seen:
            seen.add(k)
            print("SYNC:", x.filename, x.lineno, k, flush=True)
    print(f"sync warnings in one step: {len(w)}", flush=True)
    n = 20
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {(t1 - t0) / n * 1e3:.3f} ms/step, end-to-end {(t2 - t0) / n * 1e3:.3f} ms/step", flush=True)
    # host time of each phase (device idle-waiting excluded: sync before each phase)
    ph = {"fwd": 0.0, "loss_bwd": 0.0, "opt": 0.0}
    for i in range(n):
        b = bs[i % len(bs)]
        torch.cuda.synchronize()
        a = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        out, _, _ = model(*b.model_args())
        c = time.perf_counter()
        loss_fn(out, b.targets).backward()
        d = time.perf_counter()
        opt.step()
        e = time.perf_counter()
        ph["fwd"] += c - a
        ph["loss_bwd"] += d - c
        ph["opt"] += e - d
    print({k: round(v / n * 1e3, 3) for k, v in ph.items()}, "ms host per phase", flush=True)


if __name__ == "__main__":
    main()
