"""The hop's roofline-size and in-step figures per config, as bench.py computes them.

usage: python tools/hop_cfg_micro.py [--configs c4,c5] [--no-roofline]
One JSON line per config: roofline fwd/bwd (HIP events, ~4M-atom tiled graph) and the in-step
fwd/bwd at the config's own batch (graph-replayed launches). Run once per AIMX_HOP_* setting
(the launcher reads its knobs once per process) for an A/B.
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
    ap.add_argument("--configs", default="c4,c5")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-in-step", action="store_true")
    ap.add_argument("--hidden", type=int, default=0, help="override hidden (D = int(0.3 * hidden)) for width probes")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("AIMX_"))
    for c in a.configs.split(","):
        cfg = bench.CONFIGS[c]
        probe = bench.make_batches(cfg, 1, 99, dev)[0]
        hidden = a.hidden or cfg["hidden"]
        rec = {"config": c, "env": tag, "D": int(0.3 * hidden)}
        if not a.no_in_step:
            rec["in_step"] = bench.hop_in_step(probe, cfg["hops"], hidden, dev)
        if not a.no_roofline:
            r = bench.hop_roofline(probe, cfg["hops"], dev, hidden)
            rec["roofline"] = {"fwd_ms": r["ms_per_launch"], "fwd_frac": r["frac"], "bwd_us": r["bwd"]["us_per_launch"],
                               "bwd_frac": r["bwd"]["frac"], "atoms": r["atoms"], "edges": r["edges"], "D": r["D"]}
        print(json.dumps(rec), flush=True)
        del probe
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
