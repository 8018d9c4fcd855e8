"""Phase timestamps of the weight-resident MLP forward (diagnostics build: make
CXXFLAGS+=-DAIMX_MLPW_TRACE into AIMX_LIB_PATH): workgroup 0's microseconds for weight staging, the
row-chunk load and each GEMM phase, on a c2 forward and backward (backward: start, fill, dg copy,
then the dV and dA phases of each block)."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]


def main():
    import bench
    from aimx import _lib
    lib = _lib.load()
    lib.aimx_mlpw_trace_read.argtypes = [ctypes.c_void_p]
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    dev = torch.device("cuda")
    m = bench.build_model(cfg, dev)
    from aimx import autograph
    autograph.enable(m, False)  # eager launches (the stamps come from the kernels either way)
    b = bench.make_batches(cfg, 1, 5, dev)[0]
    for _ in range(5):
        out, _, _ = m(*b.model_args())
        out.sum().backward()
        m.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    buf = (ctypes.c_longlong * 64)()
    lib.aimx_mlpw_trace_read(ctypes.addressof(buf))
    t = list(buf)
    fw = [v for v in t[:32] if v]
    bw = [v for v in t[32:63] if v]
    print(json.dumps({"fwd_phases_us": [round((b_ - a) / 100.0, 2) for a, b_ in zip(fw, fw[1:])],
                      "fwd_total_us": round((t[63] - fw[0]) / 100.0, 2) if t[63] and fw else None,
                      "bwd_phases_us": [round((b_ - a) / 100.0, 2) for a, b_ in zip(bw, bw[1:])]}))

if __name__ == "__main__":
    main()
