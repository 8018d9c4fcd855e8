"""Feeder throughput with no step consuming it: batches per second the bench feed can produce
(native store or HDF5 stream), and its per-stage times, against the step time it must hide under.

  python tools/feed_rate.py --config c2 --feed stream --batches 400 --threads 8
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--feed", default="stream", choices=["native", "stream"])
    ap.add_argument("--batches", type=int, default=400)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--read-threads", type=int, default=None)
    ap.add_argument("--stream-mols", type=int, default=200_000)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    if a.feed == "native":
        it = bench.native_feeder(cfg, 0, dev, a.threads, True)
    else:
        it = bench.stream_feeder(cfg, 0, 1, dev, a.threads, True, a.stream_mols, read_threads=a.read_threads)
    for _ in range(20):
        next(it)
    torch.cuda.synchronize()
    it.reset_stats()
    t0 = time.perf_counter()
    for _ in range(a.batches):
        next(it)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"config": a.config, "feed": a.feed, "threads": a.threads, "read_threads": a.read_threads, "ms_per_batch": round(dt * 1e3 / a.batches, 4),
                      "stages": it.stats(), "stream_file": bench.STREAM_INFO or None}))


if __name__ == "__main__":
    main()
