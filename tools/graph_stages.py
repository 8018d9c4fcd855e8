"""Per-operator HIP-graph replay checks on CHANGING static inputs (batch 0, 1, 0).

Each stage captures one operator (forward + backward where it has one) with the GraphPlan built
inside the graph, replays it after copying a different padded batch into the static inputs, and
compares every output and gradient with an eager run on the same batch (exact equality expected:
the kernels are deterministic). Run one stage per process, least risky first:
  plan   CSR construction only (no backward kernels)
  embed  embedding gather + projection GEMM, forward + backward
  pool   attention pool forward + backward
  stack  message-passing stack forward + backward (eval, no dropout)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import bench  # noqa: E402
from aimx import ops  # noqa: E402
from aimx.plan import GraphPlan  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


stage = sys.argv[1]
cfgname = sys.argv[2] if len(sys.argv) > 2 else "c1"
cfg = bench.CONFIGS[cfgname]
dev = torch.device("cuda", 0)
batches = bench.make_batches(cfg, 2, 1234, dev, pad=True)
static = batches[0].clone()
H = cfg["hops"]
n = static.num_atoms
G = static.num_graphs
torch.manual_seed(0)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())


def make_plan():
    return GraphPlan(n, H, edges=static.edges, batch=static.batch, num_graphs=G)


if stage == "plan":
    def fn():
        p = make_plan()
        return [p.fwd.rowptr, p.fwd.col, p.bwd.rowptr, p.bwd.col, p.graph.rowptr, p.graph.col, p.status]
    leaves = []
elif stage == "embed":
    tables = [torch.randn(r, 64, device=dev, requires_grad=True) for r in (119, 9, 7, 7)]
    Wp = torch.randn(128, 256, device=dev, requires_grad=True)
    bp = torch.randn(128, device=dev, requires_grad=True)
    wout = torch.randn(n, 128, device=dev)
    leaves = tables + [Wp, bp]

    def fn():
        y = ops.embed_project([static.atom_features[k] for k in bench.adata.FEATURE_KEYS], tables, Wp, bp, "silu")
        (y * wout).sum().backward()
        return [y.detach()]
elif stage == "pool":
    xp = torch.randn(n, 128, device=dev, requires_grad=True)
    Wa = torch.randn(4, 128, device=dev, requires_grad=True)
    ba = torch.randn(4, device=dev, requires_grad=True)
    tau = torch.tensor(1.0, device=dev, requires_grad=True)
    wout = torch.randn(G, 128, device=dev)
    leaves = [xp, Wa, ba, tau]

    def fn():
        p = make_plan()
        pooled, attn = ops.attention_pool(p, xp, Wa, ba, tau)
        (pooled * wout).sum().backward()
        return [pooled.detach(), attn.detach()]
elif stage == "stack":
    from models import GNN
    m = GNN(bench.FS, cfg["hidden"], 1, num_shells=H).to(dev).eval()
    d = int(0.3 * cfg["hidden"])
    xs = torch.randn(n, d, device=dev, requires_grad=True)
    wout = torch.randn(n, d, device=dev)
    leaves = [xs] + list(m.message_passing_layers.parameters())

    def fn():
        p = make_plan()
        params = []
        for layer in m.message_passing_layers:
            params += layer._aimx_params()
        y = ops.message_passing_stack(p, xs, params, num_hops=H, num_layers=len(m.message_passing_layers),
                                      num_mlp=2, act="silu")
        (y * wout).sum().backward()
        return [y.detach()]
else:
    raise SystemExit(f"unknown stage {stage}")


def grads():
    return [lf.grad.clone() if lf.grad is not None else None for lf in leaves]


def zero():
    for lf in leaves:
        lf.grad = None


ref = []
with torch.cuda.stream(side):
    for b in batches:
        static.copy_(b)
        zero()
        outs = [o.clone() for o in fn()]
        ref.append((outs, grads()))
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
log(stage, "eager ok")
static.copy_(batches[0])
zero()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    outs = fn()
log(stage, "captured")
for i in (0, 1, 0):
    static.copy_(batches[i])
    g.replay()
    torch.cuda.synchronize()
    d_out = [float((a.double() - b.double()).abs().max()) if a.numel() else 0.0 for a, b in zip(outs, ref[i][0])]
    d_grad = [float((lf.grad - r).abs().max()) if r is not None else -1.0 for lf, r in zip(leaves, ref[i][1])]
    log(stage, "replay batch", i, "out diffs", d_out, "grad diffs", d_grad)
log(stage, "done")
