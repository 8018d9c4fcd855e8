"""cProfile of the eager (no-graph) c2 train step: where the host time of the drop-in path goes."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    batches = bench.make_batches(cfg, 4, 1234, dev)
    model = bench.build_model(cfg, dev)
    from aimx.optim import FusedAdam
    from models import L1Loss
    loss_fn, opt, B = L1Loss(), FusedAdam(model.parameters(), lr=2.5e-4, max_grad_norm=1.0), cfg["batch"]

    def step(i):
        b = batches[i % len(batches)]
        opt.zero_grad(set_to_none=True)
        out, _, _ = model(*b.model_args())
        loss = loss_fn(out[:B], b.targets[:B])
        loss.backward()
        opt.step()

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    n = 40
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    torch.cuda.synchronize()
    print(f"eager {cfg}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms/step", flush=True)
    pr = cProfile.Profile()
    with torch.autograd.set_multithreading_enabled(False):  # backward on this thread: profiled too
        pr.enable()
        for i in range(n):
            step(i)
        torch.cuda.synchronize()
        pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumtime").print_stats(40)


if __name__ == "__main__":
    main()
