"""HDF5 stream read rate (aimx_h5_read_store): molecules per second for shuffled 16384-molecule
chunks of a synthetic stream file in the reference format, per thread count, on this host.

  python tools/h5_read_rate.py --source qm9 --mols 200000 --threads 1 4 8 16
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "aimnet-x2d_amd"))
from aimx import h5  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--source", default="qm9")
    ap.add_argument("--mols", type=int, default=200_000)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4, 8, 16])
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--path", default=None)
    a = ap.parse_args()
    path = a.path or os.path.join(os.environ.get("TMPDIR", "/tmp"), f"aimx_rate_{a.source}_{a.hops}h_{a.mols}.h5")
    if not os.path.exists(path):
        t0 = time.perf_counter()
        h5.make_synthetic_stream(path + ".part", a.mols, a.source, a.hops, 1, seed=0, workers=16)
        os.replace(path + ".part", path)
        print(f"wrote {a.mols} molecules in {time.perf_counter() - t0:.1f} s ({os.path.getsize(path) / 1e9:.2f} GB)",
              flush=True)
    s = h5.HDF5MolecularStream(path, shuffle=True, n_hops=a.hops, n_tasks=1)
    pos = s.positions(0)
    for th in a.threads:
        s.file.read_store(pos[:16384], a.hops, 1, th)  # warm the decode buffers
        t0 = time.perf_counter()
        for c in range(a.chunks):
            s.file.read_store(pos[(c + 1) * 16384:(c + 2) * 16384], a.hops, 1, th)
        dt = time.perf_counter() - t0
        print(f"{a.source} threads {th}: {a.chunks * 16384 / dt:,.0f} mol/s  direct={s.file.direct_read}", flush=True)


if __name__ == "__main__":
    main()
