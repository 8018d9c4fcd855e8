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

    # the parity test's exact sequence (forward + backward, modes alternating): which run departs?
    w = torch.randn(n, d, device=dev)
    torch.manual_seed(1)
    ls = [ShellConvolutionLayer(d, d, num_hops=hops).to(dev) for _ in range(3)]
    params = [p for l in ls for p in l._aimx_params()]
    runs = []
    from aimx import _lib

    def state():
        d = {"x": x, "w": w, "fwd.rowptr": plan.fwd.rowptr, "fwd.col": plan.fwd.col, "bwd.rowptr": plan.bwd.rowptr,
             "bwd.col": plan.bwd.col, "counters": _lib.counters(dev), "batch": plan._keep[-1], "seed": seed}
        seg = plan.row_seg()
        d.update({f"param{i}": p for i, p in enumerate(params)})
        return {k: v.detach().clone() for k, v in d.items()}, seg

    snap, seg0 = state()
    for mode, rt in (("0", None), ("0", None), ("0", None), ("1", None), ("0", None), ("1", "1"), ("0", None),
                     ("1", None)):
        os.environ["AIMX_MLPS"] = mode
        if rt:
            os.environ["AIMX_MLPS_RT"] = rt
        xs = x.clone().requires_grad_()
        ps = [p.detach().clone().requires_grad_() for p in params]
        y = ops.message_passing_stack(plan, xs, ps, num_hops=hops, num_layers=3, num_mlp=2, act="silu", training=True,
                                      drop_p=0.05, drop_seed=seed)
        y0 = y.detach().clone()
        torch.cuda.synchronize()
        (y * w).sum().backward()
        torch.cuda.synchronize()
        os.environ.pop("AIMX_MLPS_RT", None)
        runs.append((mode, rt, y0, xs.grad.clone(), [q.grad.clone() for q in ps]))
        r0 = runs[0]
        ey = ((y0 - r0[2]).norm() / r0[2].norm()).item()
        ex = ((xs.grad - r0[3]).norm() / r0[3].norm()).item()
        ep = max(((a - b).norm() / b.norm().clamp_min(1e-30)).item() for a, b in zip(runs[-1][4], r0[4]))
        print(f"seq run {len(runs) - 1} mode={mode} rt={rt}: y {ey:.2e} dx {ex:.2e} dparams max {ep:.2e}", flush=True)
        now, seg1 = state()
        changed = [k for k in snap if not torch.equal(now[k], snap[k])]
        nz = int((now["counters"] != 0).sum())
        print(f"   changed since start: {changed}; nonzero counters {nz}; row_seg {seg0 == seg1}", flush=True)
        if changed:
            for k in changed:
                dif = (now[k] != snap[k]).nonzero().flatten()
                print(f"   {k}: {dif.numel()} elements differ, first at {dif[:8].tolist()}", flush=True)
            snap = now
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
