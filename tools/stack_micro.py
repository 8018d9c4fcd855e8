"""Time the message-passing stack forward and backward alone (c2-sized QM9 batch)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import bench  # noqa: E402
from aimx import ops  # noqa: E402
from aimx.plan import GraphPlan  # noqa: E402
from models import GNN  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
dev = torch.device("cuda", 0)
b = bench.make_batches(cfg, 1, 1234, dev)[0]
m = GNN(bench.FS, cfg["hidden"], 1, num_shells=cfg["hops"]).to(dev).eval()
d = int(0.3 * cfg["hidden"])
plan = GraphPlan(b.num_atoms, cfg["hops"], edges=b.edges, batch=b.batch, num_graphs=b.num_graphs)
x = torch.randn(b.num_atoms, d, device=dev, requires_grad=True)
params = []
for layer in m.message_passing_layers:
    params += [p.detach().requires_grad_() for p in layer._aimx_params()]


def fwd():
    return ops.message_passing_stack(plan, x, params, num_hops=cfg["hops"], num_layers=3, num_mlp=2, act="silu")


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e3


with torch.no_grad():
    tf = timeit(fwd)
y = fwd()
g = torch.randn_like(y)
tb = timeit(lambda: torch.autograd.grad(y, [x] + params, g, retain_graph=True))
print(f"stack fwd {tf:8.1f} us   bwd {tb:8.1f} us   (N={b.num_atoms}, D={d})")
