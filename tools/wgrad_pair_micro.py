"""Two c2 long-K weight gradients (concat_self_other and embedding projection: dW = dY^T X,
256 x 257 with the bias column, K = 9170) as two single launches (the step's k_wgrad path) vs ONE
grouped launch (ops.wgrad_grouped), graph-timed."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd"), os.path.join(ROOT, "tools")]
from aimx import ops  # noqa: E402


def bench(fn, it=20):
    """us per call: a HIP graph of `it` back-to-back calls, replayed 5 times."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(5):
        g.replay()
    t1.record()
    t1.synchronize()
    return t0.elapsed_time(t1) / (5 * it) * 1e3

dev = "cuda"
K, M, N = 9170, 256, 256
dys = [torch.randn(K, M, device=dev) for _ in range(2)]
xs = [torch.randn(K, N, device=dev) for _ in range(2)]
Ws = [torch.randn(M, N, device=dev) for _ in range(2)]
dWs = [torch.empty(M, N, device=dev) for _ in range(2)]
dbs = [torch.empty(M, device=dev) for _ in range(2)]
dxs = [torch.empty(K, N, device=dev) for _ in range(2)]


def single():
    for i in range(2):
        ops.gemm_linear_bwd(dys[i], M, xs[i], N, Ws[i], None, dWs[i], dbs[i], ops.PREC_FP32)


def grouped():
    ops.wgrad_grouped([(dys[i], xs[i], dWs[i], dbs[i]) for i in range(2)])


for name, fn in (("two single launches", single), ("one grouped launch", grouped)):
    print(f"{name:22s} {bench(fn, it=20):7.1f} us", flush=True)
