"""Where the weight-streamed MLP chain (AIMX_MLPS=1) departs from the per-GEMM path: stack forward
over a config-shaped batch in both modes, the error by variant (layers, blocks, dropout, chunk rows)
and, for the worst variant, by column fragment and by row chunk.

usage: python tools/debug_mlps.py [hidden hops mols]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "aimnet-x2d_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main():
    hidden, hops, mols = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (512, 3, 512)))
    import aimx
    from aimx import ops
    from aimx import data as adata
    from aimx.plan import GraphPlan
    from aimx.synth import synth_molecules
    from models.layers import ShellConvolutionLayer
    aimx.load()
    dev = "cuda"
    torch.manual_seed(0)
    col = adata.collate(synth_molecules(mols, seed=0), hops)
    edges = torch.from_numpy(col["edges"]).to(dev)
    batch = torch.from_numpy(col["batch"]).to(dev)
    n, d = batch.shape[0], int(0.3 * hidden)
    plan = GraphPlan(n, hops, edges=edges, batch=batch, num_graphs=mols)
    x = torch.randn(n, d, device=dev)
    seed = torch.tensor([4321], device=dev)
    print(f"N={n} D={d}", flush=True)

    def run(mode, layers, nm, train, rt=None):
        os.environ["AIMX_MLPS"] = mode
        if rt is not None:
            os.environ["AIMX_MLPS_RT"] = str(rt)
        else:
            os.environ.pop("AIMX_MLPS_RT", None)
        torch.manual_seed(1)
        ls = [ShellConvolutionLayer(d, d, num_hops=hops, num_mlp_layers=nm).to(dev) for _ in range(layers)]
        ps = [p.detach().clone() for l in ls for p in l._aimx_params()]
        with torch.no_grad():
            y = ops.message_passing_stack(plan, x, ps, num_hops=hops, num_layers=layers, num_mlp=nm, act="silu",
                                          training=train, drop_p=0.05 if train else 0.0, drop_seed=seed)
        torch.cuda.synchronize()
        return y

    worst = None
    for layers, nm in ((1, 1), (1, 2), (3, 2)):
        for train in (False, True):
            for rt in (None, 1):
                ref = run("0", layers, nm, train)
                errs = []
                for rep in range(3):
                    y = run("1", layers, nm, train, rt)
                    errs.append(((y - ref).norm() / ref.norm()).item())
                ref2 = run("0", layers, nm, train)
                e0 = ((ref2 - ref).norm() / ref.norm()).item()
                print(f"layers={layers} nm={nm} train={train} rt={rt}: rel err {['%.2e' % e for e in errs]} "
                      f"(per-GEMM rerun {e0:.2e})", flush=True)
                if worst is None or max(errs) > worst[0]:
                    worst = (max(errs), layers, train, rt, y, ref)
    e, layers, train, rt, y, ref = worst
    print(f"worst: layers={layers} train={train} rt={rt} err={e:.3e}")
    diff = (y - ref).abs()
    scale = ref.abs().mean().item()
    for f in range((d + 15) // 16):
        c = diff[:, 16 * f:16 * f + 16]
        print(f"  frag {f:2d} cols {16 * f:4d}..{min(d, 16 * f + 16) - 1:4d}: max {c.max().item() / scale:.2e} "
              f"mean {c.mean().item() / scale:.2e}")
    rows = diff.max(dim=1).values / scale
    bad = (rows > 1e-3).nonzero().flatten()
    print(f"  rows with err > 1e-3: {bad.numel()} of {n}; first {bad[:20].tolist()}")
    if bad.numel():
        print(f"  row mod 16 histogram: {torch.bincount(bad % 16, minlength=16).tolist()}")
        print(f"  row mod 80 histogram (first 20 bins): {torch.bincount(bad % 80, minlength=80)[:20].tolist()}")


if __name__ == "__main__":
    main()
