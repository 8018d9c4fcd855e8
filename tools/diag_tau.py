import sys, os, numpy as np, torch
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "aimnet-x2d_amd"), os.path.join(os.getcwd(), "tests")]
import aimx; aimx.load()
from models.pooling import MultiHeadAttentionPoolingLayer
from oracle import model as om
def run(C, H, sizes, seed, mean=3.0):
    g = torch.Generator().manual_seed(seed)
    batch = torch.cat([torch.full((s,), i, dtype=torch.long) for i, s in enumerate(sizes)])
    n = batch.numel()
    x = mean + torch.randn(n, C, generator=g)
    pool = MultiHeadAttentionPoolingLayer(C, num_heads=H, initial_temperature=0.7)
    with torch.no_grad():
        for lin in pool.attention_weights:
            lin.weight.copy_(torch.randn(1, C, generator=g) * 0.1); lin.bias.copy_(torch.randn(1, generator=g))
    params = {k: v.detach().clone() for k, v in pool.state_dict().items()}
    wp = torch.randn(len(sizes), C, generator=g); wa = torch.randn(H, n, generator=g)
    pool = pool.cuda(); xd = x.cuda().requires_grad_()
    pooled, attn = pool(xd, batch.cuda())
    ((pooled * wp.cuda()).sum() + (attn * wa.cuda()).sum()).backward()
    ours = pool.temperature.grad.item()
    res = {}
    for dt in (torch.float32, torch.float64):
        pd = {"pool." + k: v.detach().to(dt).requires_grad_() for k, v in params.items()}
        xr = x.detach().to(dt).requires_grad_()
        pp, aa = om.attention_pool(pd, "pool.", xr, batch, H, len(sizes))
        ((pp * wp.to(dt)).sum() + (aa * wa.to(dt)).sum()).backward()
        res[dt] = pd["pool.temperature"].grad.item()
    r64 = res[torch.float64]
    return abs(ours - r64) / abs(r64), abs(res[torch.float32] - r64) / abs(r64)
small = [1, 2, 7, 18, 29, 31, 32, 33, 40, 47, 48, 49, 64, 65, 100, 128, 3]
large = [129, 300, 600]
for C, H in [(1024, 8), (1024, 4), (512, 8), (256, 4)]:
    for name, sz in [("small", small), ("large", large), ("all", small + large)]:
        for seed in (C * 10 + H, 1, 2):
            e, e32 = run(C, H, sz, seed)
            print(C, H, name, seed, f"ours {e:.2e} ref32 {e32:.2e}")
