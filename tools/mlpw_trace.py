"""Phase timestamps of the weight-resident MLP forward (diagnostics build: make
CXXFLAGS+=-DAIMX_MLPW_TRACE into AIMX_LIB_PATH): workgroup 0's microseconds for weight staging, the
row-chunk load and each GEMM phase, on a c2 forward."""
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
    b = bench.make_batches(cfg, 1, 5, dev)[0]
    for _ in range(5):
        with torch.no_grad():
            m(*b.model_args())
    torch.cuda.synchronize()
    buf = (ctypes.c_longlong * 64)()
    lib.aimx_mlpw_trace_read(ctypes.addressof(buf))
    t = list(buf)
    st = [v for v in t[:63] if v]
    print(json.dumps({"phases_us": [round((b_ - a) / 100.0, 2) for a, b_ in zip(st, st[1:])],
                      "total_us": round((t[63] - st[0]) / 100.0, 2) if t[63] and st else None}))


if __name__ == "__main__":
    main()
