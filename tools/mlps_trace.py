"""Phase timeline of the weight-streamed node-update MLP (k_mlps_fwd / k_mlps_bwd) from in-kernel
stamps: a diagnostics build of mlp.hip (-DAIMX_MLPS_TRACE, lib/libaimx_mlps_trace.so) records, for
workgroups 0 and 77, each wave's wall clock (100 MHz) at kernel entry, after the bias / zero fill,
after the chunk load, and per GEMM of the chain after its k loop, after its epilogue and after the
refill + LDS barrier. Runs one c4- or c5-shaped stack forward + backward and prints, per traced
workgroup, each phase's span over the waves (min / max of the per-wave durations, in us).

usage: python tools/mlps_trace.py [c4|c5]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("AIMX_LIB_PATH", os.path.join(ROOT, "aimnet-x2d_amd", "lib", "libaimx_mlps_trace.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

SHAPES = {"c4": (512, 3, 512), "c5": (1024, 6, 256)}


def main():
    import numpy as np
    import torch
    import aimx
    from aimx import _lib, ops
    from aimx import data as adata
    from aimx.plan import GraphPlan
    from aimx.synth import synth_molecules
    from models.layers import ShellConvolutionLayer
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
    buf = np.zeros((2, 2, 12, 24), np.int64)
    rc = _lib.load().aimx_mlps_trace_read(buf.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise SystemExit("trace read failed (is AIMX_LIB_PATH the -DAIMX_MLPS_TRACE build?)")
    print(f"{cfg}: N={n} D={d} (last forward launch = layer 2, last backward = layer 0); us per phase, "
          "min..max over the waves")
    for dr, name in ((0, "fwd"), (1, "bwd")):
        for slot, wg in ((0, 0), (1, 77)):
            t = buf[dr, slot]
            waves = [w for w in range(12) if t[w, 0] != 0]
            if not waves:
                continue
            labels = ["init", "chunk load"] + [f"g{ph} {part}" for ph in range(4) for part in ("kloop", "epilogue",
                                                                                              "refill+sync")]
            t0 = min(t[w, 0] for w in waves)
            end = max(t[w, 14] for w in waves)
            print(f"== {name} workgroup {wg}: {len(waves)} waves, span {(end - t0) / 100:.2f} us")
            for k, lab in enumerate(labels, start=1):
                dur = [(t[w, k] - t[w, k - 1]) / 100 for w in waves]
                at = (min(t[w, k] for w in waves) - t0) / 100
                print(f"  {lab:18s} {min(dur):7.2f} .. {max(dur):7.2f}   (first wave done at {at:7.2f})")


if __name__ == "__main__":
    main()
