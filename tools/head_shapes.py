"""Graph-timed fused head forward alone (ops.head, eval) over F and block count: separates the
per-layer cost from fixed costs."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
from head_micro import timed  # noqa: E402


def main():
    from aimx import ops
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    for F in (128, 256):
        for nb in (1, 3, 6):
            mk = lambda *s: (torch.randn(*s, generator=g) * 0.05).to(dev)  # noqa: E731
            x = mk(520, F)
            blocks = [(mk(F, F), mk(F), mk(F, F), mk(F)) for _ in range(nb)]
            args = (x, mk(F, F), mk(F), blocks, mk(F, F), mk(F), mk(1, 2 * F), mk(1))

            def fwd():
                with torch.no_grad():
                    ops.head(*args, act="silu", skips=[False] * nb)
            print(json.dumps({"F": F, "nb": nb, "gemms": 2 * nb + 3, "us": timed(fwd)}), flush=True)


if __name__ == "__main__":
    main()
