"""Staged HIP-graph replay check: which phase of the train step misbehaves on a changed batch.

Stages (each logged and flushed; the first failure ends the process):
  A  eager fwd+bwd on every padded batch (data check, side stream)
  B  capture forward only; replay batch 0, 0, 1, 0 and compare with eager forward outputs
  C  capture forward+backward; replay 0, 1, 0 and compare gradients with eager
  D  capture forward+backward+clip+Adam; replay 0, 1, 0
"""
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


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


cfgname = sys.argv[1] if len(sys.argv) > 1 else "c1"
stages = sys.argv[2] if len(sys.argv) > 2 else "ABCD"
cfg = bench.CONFIGS[cfgname]
dev = torch.device("cuda", 0)
batches = bench.make_batches(cfg, 2, 1234, dev, pad=True)
log("batches", [b.num_atoms for b in batches], [b.real_atoms for b in batches])
model = bench.build_model(cfg, dev).eval()  # dropout off: replay must equal eager exactly
B = cfg["batch"]
loss_fn = torch.nn.L1Loss()
static = batches[0].clone()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())


def fwd():
    return model(*static.model_args())[0]


def fwd_bwd():
    out = fwd()
    loss = loss_fn(out[:B], static.targets[:B])
    loss.backward()
    return out.detach()


def grads():
    return torch.cat([p.grad.reshape(-1) for p in model.parameters() if p.grad is not None])


ref_out, ref_grad = [], []
with torch.cuda.stream(side):
    for i, b in enumerate(batches):
        static.copy_(b)
        model.zero_grad(set_to_none=True)
        ref_out.append(fwd_bwd().clone())
        ref_grad.append(grads().clone())
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
log("A eager ok on all batches", [float(o.abs().sum()) for o in ref_out])
if "A" == stages:
    sys.exit(0)


def replay_check(name, g, out, order, check_grad=False):
    for i in order:
        static.copy_(batches[i])
        g.replay()
        torch.cuda.synchronize()
        d = float((out - ref_out[i]).abs().max())
        msg = f"{name} replay batch {i}: max|out-eager| {d:.3e}"
        if check_grad:
            dg = float((grads() - ref_grad[i]).abs().max())
            msg += f" max|grad-eager| {dg:.3e}"
        log(msg)


if "B" in stages:
    static.copy_(batches[0])
    gB = torch.cuda.CUDAGraph()
    with torch.no_grad():
        with torch.cuda.stream(side):
            fwd()
        torch.cuda.synchronize()
        with torch.cuda.graph(gB):
            outB = fwd()
    log("B captured")
    replay_check("B", gB, outB, [0, 0, 1, 0])
    del gB, outB

if "C" in stages:
    static.copy_(batches[0])
    model.zero_grad(set_to_none=True)
    with torch.cuda.stream(side):
        fwd_bwd()
    torch.cuda.synchronize()
    model.zero_grad(set_to_none=True)
    gC = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gC):
        outC = fwd_bwd()
    log("C captured")
    replay_check("C", gC, outC, [0, 1, 0], check_grad=True)
    del gC, outC

if "D" in stages:
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=2.5e-4, capturable=True)
    with torch.cuda.stream(side):
        for _ in range(2):
            opt.zero_grad(set_to_none=True)
            fwd_bwd()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    opt.zero_grad(set_to_none=True)
    gD = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gD):
        fwd_bwd()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
    log("D captured")
    for i in (0, 1, 0):
        static.copy_(batches[i])
        gD.replay()
        torch.cuda.synchronize()
        log("D replay batch", i, "ok")
log("done")
