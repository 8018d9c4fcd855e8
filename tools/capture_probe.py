"""Capture each aimx operator alone in a HIP graph (progress flushed) to find capture-unsafe calls."""
import os
import sys
import time

import torch

if os.environ.get("CRASHTRACE"):
    import ctypes
    ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_crashtrace.so")).crashtrace_install()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import bench  # noqa: E402
from aimx import ops  # noqa: E402
from aimx.plan import GraphPlan  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


dev = torch.device("cuda", 0)
cfg = bench.CONFIGS["c1"]
b = bench.make_batches(cfg, 1, 1234, dev, pad=True)[0]
n = b.num_atoms
x = torch.randn(n, 38, device=dev)
W = torch.randn(76, 304 // 2, device=dev)


def cap(name, fn):
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    log(name, "eager ok")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode=os.environ.get("CAPMODE", "global")):
        fn()
    log(name, "captured")
    g.replay()
    torch.cuda.synchronize()
    log(name, "replayed")


which = sys.argv[1:] or ["plan", "hop", "gemm", "stack", "pool", "embed"]
if "plan" in which:
    cap("plan", lambda: GraphPlan(n, 3, edges=b.edges, batch=b.batch, num_graphs=b.num_graphs))
plan = GraphPlan(n, 3, edges=b.edges, batch=b.batch, num_graphs=b.num_graphs)
if "hop" in which:
    cap("hop", lambda: ops.hop(plan, x))
if "gemm" in which:
    Wl = torch.randn(38, 38, device=dev)
    bl = torch.randn(38, device=dev)
    cap("gemm", lambda: ops.linear(x, Wl, bl, "silu"))
if "stack" in which:
    from models import GNN
    m = GNN(bench.FS, 128, 1).to(dev)
    params = []
    for l in m.message_passing_layers:
        params += l._aimx_params()
    cap("stack", lambda: ops.message_passing_stack(plan, x, [p.detach() for p in params], num_hops=3, num_layers=3,
                                                   num_mlp=2, act="silu"))
if "pool" in which:
    xp = torch.randn(n, 128, device=dev)
    Wp = torch.randn(4, 128, device=dev)
    bp = torch.randn(4, device=dev)
    tau = torch.tensor(1.0, device=dev)
    cap("pool", lambda: ops.attention_pool(plan, xp, Wp, bp, tau))
if "embed" in which:
    tables = [torch.randn(r, 64, device=dev) for r in (119, 9, 7, 7)]
    Wp = torch.randn(128, 256, device=dev)
    bp = torch.randn(128, device=dev)
    cap("embed", lambda: ops.embed_project([b.atom_features[k] for k in bench.adata.FEATURE_KEYS], tables, Wp, bp,
                                           "silu"))
xr = x.clone().requires_grad_()
if "hop_b" in which:
    cap("hop_b", lambda: ops.hop(plan, xr).sum().backward())
if "gemm_b" in which:
    Wl = torch.randn(38, 38, device=dev, requires_grad=True)
    bl = torch.randn(38, device=dev, requires_grad=True)
    cap("gemm_b", lambda: ops.linear(xr, Wl, bl, "silu").sum().backward())
if "stack_b" in which:
    from models import GNN
    m = GNN(bench.FS, 128, 1).to(dev)

    def stack_b():
        # params are built inside the captured region: autograd nodes created on another stream
        # (e.g. the legacy default stream) must not be part of a captured backward
        params = []
        for l in m.message_passing_layers:
            params += l._aimx_params()
        ops.message_passing_stack(plan, xr, params, num_hops=3, num_layers=3, num_mlp=2, act="silu").sum().backward()
    cap("stack_b", stack_b)
if "pool_b" in which:
    xp = torch.randn(n, 128, device=dev, requires_grad=True)
    Wp = torch.randn(4, 128, device=dev, requires_grad=True)
    bp = torch.randn(4, device=dev, requires_grad=True)
    tau = torch.tensor(1.0, device=dev, requires_grad=True)
    cap("pool_b", lambda: ops.attention_pool(plan, xp, Wp, bp, tau)[0].sum().backward())
if "embed_b" in which:
    tables = [torch.randn(r, 64, device=dev, requires_grad=True) for r in (119, 9, 7, 7)]
    Wp = torch.randn(128, 256, device=dev, requires_grad=True)
    bp = torch.randn(128, device=dev, requires_grad=True)
    cap("embed_b", lambda: ops.embed_project([b.atom_features[k] for k in bench.adata.FEATURE_KEYS], tables, Wp, bp,
                                             "silu").sum().backward())
log("all done")
