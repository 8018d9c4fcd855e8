"""Where k_wgrad_lds's waves spend their time: a diagnostics build of gemm.hip (-DAIMX_WB_TRACE,
lib/libaimx_wb_trace.so) sums, per wave of workgroups 0 / 777 / 2222 / 4444 of the last launch, the
shader clocks spent in put (which first waits for the fill's global loads), fetch (load issue),
compute (LDS reads + MFMAs) and the fill barriers, against the wave's whole loop. Runs a c4- or
c5-shaped stack forward + backward (the stack's grouped weight gradients are the last launch).

usage: python tools/wgrad_trace.py [c4|c5]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("AIMX_LIB_PATH", os.path.join(ROOT, "aimnet-x2d_amd", "lib", "libaimx_wb_trace.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd"), os.path.join(ROOT, "tools")]


def main():
    import numpy as np
    import torch
    import aimx
    from aimx import _lib, ops
    from aimx import data as adata
    from aimx.plan import GraphPlan
    from aimx.synth import synth_molecules
    from models.layers import ShellConvolutionLayer
    from mlps_trace import SHAPES
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    hidden, hops, mols = SHAPES[cfg]
    aimx.load()
    dev = "cuda"
    torch.manual_seed(0)
    col = adata.collate(synth_molecules(mols, seed=0), hops)
    edges = torch.from_numpy(col["edges"]).to(dev)
    batch = torch.from_numpy(col["batch"]).to(dev)
    n, d = batch.shape[0], int(0.3 * hidden)
    plan = GraphPlan(n, hops, edges=edges, batch=batch, num_graphs=mols)
    x = torch.randn(n, d, device=dev, requires_grad=True)
    ls = [ShellConvolutionLayer(d, d, num_hops=hops).to(dev) for _ in range(3)]
    params = [p for l in ls for p in l._aimx_params()]
    seed = torch.tensor([4321], device=dev)
    for _ in range(3):
        y = ops.message_passing_stack(plan, x, params, num_hops=hops, num_layers=3, num_mlp=2, act="silu",
                                      training=True, drop_p=0.05, drop_seed=seed)
        y.sum().backward()
    torch.cuda.synchronize()
    buf = np.zeros((4, 10, 5), np.int64)
    if _lib.load().aimx_wb_trace_read(buf.ctypes.data_as(ctypes.c_void_p)) != 0:
        raise SystemExit("trace read failed (is AIMX_LIB_PATH the -DAIMX_WB_TRACE build?)")
    print(f"{cfg}: N={n} D={d}; per wave: shader clocks (k) in put / fetch / compute / barrier, and % of its loop")
    for slot, wg in enumerate((0, 777, 2222, 4444)):
        rows = [buf[slot, w] for w in range(10) if buf[slot, w, 4] > 0]
        if not rows:
            continue
        tot = np.mean([r[4] for r in rows])
        parts = np.mean([r[:4] for r in rows], axis=0)
        print(f"  workgroup {wg:5d} ({len(rows)} waves): loop {tot / 1e3:8.1f}k  put {parts[0] / 1e3:7.1f}k "
              f"({100 * parts[0] / tot:4.1f} %)  fetch {parts[1] / 1e3:6.1f}k ({100 * parts[1] / tot:4.1f} %)  "
              f"compute {parts[2] / 1e3:7.1f}k ({100 * parts[2] / tot:4.1f} %)  barrier {parts[3] / 1e3:7.1f}k "
              f"({100 * parts[3] / tot:4.1f} %)")


if __name__ == "__main__":
    main()
