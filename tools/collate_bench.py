"""Host batch-builder throughput: native (libaimx_host.so) vs the Python restatement (aimx.data),
on the bench configs' batches. Prints one JSON line per case (molecules/s of plan+write into a
pinned DeviceBatch blob; the Python case is BFS + collate + blob packing, as bench.py uses it).

usage: python tools/collate_bench.py [--threads 1 4 8] [--seconds 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
from aimx import data as adata  # noqa: E402
from aimx import feed  # noqa: E402
from aimx.synth import QM9Asset, synth_molecules  # noqa: E402


def rate(fn, batch, seconds):
    fn()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        n += 1
    return batch * n / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4, 8])
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    asset = QM9Asset()
    syn = synth_molecules(4096, seed=1)
    cases = [("c2 qm9 B512 h3", asset, None, 512, 3), ("c3 qm9 B512 h4", asset, None, 512, 4),
             ("c4 synth40 B512 h3", None, syn, 512, 3), ("c5 synth40 B256 h6", None, syn, 256, 6)]
    pinned = torch.cuda.is_available()
    for name, qa, mols, B, hops in cases:
        n_mol = len(qa) if qa is not None else len(mols)
        idx = rng.integers(0, n_mol, B)
        pm = qa.molecules(idx) if qa is not None else [mols[i] for i in idx]

        def py():
            adata.DeviceBatch(adata.collate(pm, hops), "cpu")
        print(json.dumps({"case": name, "impl": "python aimx.data", "threads": 1,
                          "mol_per_s": round(rate(py, B, a.seconds), 1)}), flush=True)
        for cache in (0, hops):
            for t in a.threads:
                store = (feed.HostStore.from_qm9_asset(qa, precompute_hops=cache, threads=t) if qa is not None
                         else feed.HostStore.from_molecules(mols, precompute_hops=cache, threads=t))
                col = feed.HostCollator(hops, t)
                r = rate(lambda: col.collate_blob(store, idx, pinned=pinned), B, a.seconds)
                print(json.dumps({"case": name, "impl": "native" + (" cached hops" if cache else " bfs per batch"),
                                  "threads": t, "pinned": pinned, "mol_per_s": round(r, 1)}), flush=True)


if __name__ == "__main__":
    main()
