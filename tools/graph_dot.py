"""Capture the train-step graphs WITHOUT replaying them and dump their HIP graph topology (DOT).

Used to check that the captured step is a single dependency chain (one stream) and to list any
parallel branches, memset/memcpy/event nodes. Stages: B = forward only, C = forward + backward.
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import bench  # noqa: E402
from aimx import _lib  # noqa: E402
import threading  # noqa: E402

_seen = {}
_orig_stream_ptr = _lib.stream_ptr


def _spy(device=None):
    sp = _orig_stream_ptr(device)
    key = (threading.current_thread().name, sp, torch.cuda.is_current_stream_capturing())
    _seen[key] = _seen.get(key, 0) + 1
    return sp


_lib.stream_ptr = _spy
from aimx import ops as _ops  # noqa: E402
_ops.stream_ptr = _spy


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


cfgname = sys.argv[1] if len(sys.argv) > 1 else "c1"
stages = sys.argv[2] if len(sys.argv) > 2 else "BC"
out_dir = os.path.join(ROOT, "gpurun_out")
os.makedirs(out_dir, exist_ok=True)
cfg = bench.CONFIGS[cfgname]
dev = torch.device("cuda", 0)
batches = bench.make_batches(cfg, 1, 1234, dev, pad=True)
model = bench.build_model(cfg, dev).eval()
B = cfg["batch"]
static = batches[0].clone()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())


def fwd():
    return model(*static.model_args())[0]


def fwd_bwd():
    out = fwd()
    torch.nn.functional.l1_loss(out[:B], static.targets[:B]).backward()


with torch.cuda.stream(side):
    fwd_bwd()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
log("eager ok")
if "B" in stages:
    g = torch.cuda.CUDAGraph()
    g.enable_debug_mode()
    with torch.no_grad():
        with torch.cuda.graph(g):
            fwd()
    g.debug_dump(os.path.join(out_dir, f"graph_{cfgname}_B.dot"))
    log("B dumped")
    del g
if "C" in stages:
    _seen.clear()
    model.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    g.enable_debug_mode()
    with torch.cuda.graph(g):
        fwd_bwd()
    log("C streams seen by aimx launches:")
    for k, v in sorted(_seen.items(), key=str):
        log("   thread", k[0], "stream", hex(k[1]), "capturing", k[2], "calls", v)
    g.debug_dump(os.path.join(out_dir, f"graph_{cfgname}_C.dot"))
    log("C dumped")
    del g
torch.cuda.synchronize()
log("done")
