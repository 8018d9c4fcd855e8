"""The oracle pin on THIS host's CPU: for every golden fixture case, per tensor, the oracle's fp32
error against the reference's own fp32 result (the fixture) next to the reference's own fp32 error
against exact (fp64 oracle), and their ratio. The fixtures were made in the development container;
ATen's vectorised fp32 CPU kernels differ by ISA, so on another host the oracle's fp32 run moves
by a fraction of the reference's own rounding error. usage: python tools/pin_probe.py [cases...]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

from conftest import _den, _rel, fixture_refs  # noqa: E402
from golden_cases import CASES  # noqa: E402
from test_oracle_golden import oracle_run  # noqa: E402


def main():
    torch.set_num_threads(8)
    out = {"cpu": torch.backends.cpu.get_cpu_capability(), "cases": {}}
    for name in sys.argv[1:] or CASES:
        z, r32, _ = oracle_run(name, torch.float32)
        _, r64, _ = oracle_run(name, torch.float64)
        ref = fixture_refs(z)
        worst = []
        for k, v in ref.items():
            den = _den(k, r64[k], r64)
            pin, own = _rel(r32[k], v, den), _rel(v, r64[k], den)
            worst.append((pin, own, k))
        worst.sort(reverse=True)
        out["cases"][name] = {"max_pin": worst[0][0], "max_ratio": max(p / max(o, 1e-12) for p, o, _ in worst),
                              "top": [(k, p, o) for p, o, k in worst[:3]]}
        print(name, json.dumps(out["cases"][name]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
