"""Staged check of the padded-batch + HIP-graph train step (progress printed and flushed per stage)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import bench  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


cfgname = sys.argv[1] if len(sys.argv) > 1 else "c1"
stage = sys.argv[2] if len(sys.argv) > 2 else "all"
cfg = bench.CONFIGS[cfgname]
dev = torch.device("cuda", 0)
batches = bench.make_batches(cfg, 2, 1234, dev, pad=True)
log("batches", batches[0].num_atoms, batches[0].edges.shape, batches[0].num_graphs)
model = bench.build_model(cfg, dev)
B = cfg["batch"]
loss_fn = torch.nn.L1Loss()
opt = torch.optim.Adam(model.parameters(), lr=2.5e-4, capturable=True)
static = batches[0].clone()


def fwd_bwd():
    out, _, _ = model(*static.model_args())
    loss = loss_fn(out[:B], static.targets[:B])
    loss.backward()
    return loss


def clip_step():
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step()


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    opt.zero_grad(set_to_none=True)
    lv = float(fwd_bwd())  # keep no reference to the eager autograd graph
    clip_step()
torch.cuda.synchronize()
log("eager padded step ok, loss", lv)
if stage == "eager":
    sys.exit(0)
with torch.cuda.stream(side):
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        fwd_bwd()
        clip_step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
log("side-stream warmup ok")
opt.zero_grad(set_to_none=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    sl = fwd_bwd()
    clip_step()
log("captured")
for i in range(3):
    static.copy_(batches[i % 2])
    g.replay()
    torch.cuda.synchronize()
    log("replay", i, "loss", float(sl))
log("done")
