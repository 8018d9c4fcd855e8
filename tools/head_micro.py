"""Graph-timed post-pool head of the c2 model (post_pooling_projection -> ffn (3 LinearBlocks) ->
skip_transform -> cat -> output_layer -> L1 loss), forward and forward+backward, on [520, 256]."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]


def timed(fn, it=20):
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
    return round(t0.elapsed_time(t1) / (5 * it) * 1e3, 1)


def main():
    from models import GNN, L1Loss
    dev = torch.device("cuda")
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, 256, 1).to(dev).train()
    crit = L1Loss()
    xp = torch.randn(520, 256, device=dev, requires_grad=True)
    y = torch.randn(512, 1, device=dev)

    def head():
        x = m.ffn(m.post_pooling_projection(xp))
        out = m.output_layer(torch.cat([x, m.skip_transform(x)], dim=-1))
        return crit(out[:512], y)

    def fwd():
        with torch.no_grad():
            head()

    def fwdbwd():
        head().backward()

    from aimx import _lib, ops
    blocks = list(m.ffn.layers)

    def fused():
        out = ops.head(xp, m.post_pooling_projection.weight, m.post_pooling_projection.bias,
                       [(b.linear1.weight, b.linear1.bias, b.linear2.weight, b.linear2.bias) for b in blocks],
                       m.skip_transform.weight, m.skip_transform.bias, m.output_layer.weight, m.output_layer.bias,
                       act="silu", drop_p=0.05, training=True, skips=[b.use_skip for b in blocks])
        return crit(out[:512], y)

    def ffwd():
        with torch.no_grad():
            fused()

    def ffwdbwd():
        fused().backward()

    res = {"head_fwd_us": timed(fwd), "head_fwd_bwd_us": timed(fwdbwd)}
    for cfg in os.environ.get("HEAD_CLUSTERS", "1,2,4").split(","):
        S, _, W = cfg.partition("w")  # "4" or "4w8": cluster 4, 8 waves
        _lib.HEAD_CLUSTER_FORCE = int(S)
        if W:  # (tuning build only: AIMX_LIB_PATH=lib/libaimx_tune.so)
            os.environ["AIMX_HEAD_WAVES"] = W
        else:
            os.environ.pop("AIMX_HEAD_WAVES", None)
        res[f"fused_fwd_us[{cfg}]"] = timed(ffwd)
        res[f"fused_fwd_bwd_us[{cfg}]"] = timed(ffwdbwd)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
