"""Per-stage host time of one feed batch (plan / write / CSR) at a bench config, pinned or
pageable blob, over thread counts: where the batch builder's time goes.
usage: python tools/collate_stages.py [--config c4] [--threads 1,4,8,16] [--reps 30]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]
import bench  # noqa: E402
from aimx import feed  # noqa: E402
from aimx.synth import QM9Asset, synth_molecules  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    rng = np.random.default_rng(0)
    if cfg["source"] == "qm9":
        q = QM9Asset()
        store = feed.HostStore.from_arrays(q.atom_off, q.bond_off, np.stack([q.bi, q.bj], 1), q.feats,
                                           q.targets[:, :cfg["tasks"]], q.total_charge, precompute_hops=cfg["hops"],
                                           threads=8)
    else:
        mols = synth_molecules(8192, seed=0)
        store = feed.HostStore.from_molecules(mols, rng.standard_normal((len(mols), cfg["tasks"])),
                                              precompute_hops=cfg["hops"], threads=8)
    B = cfg["batch"]
    for thr in [int(t) for t in a.threads.split(",")]:
        col = feed.HostCollator(cfg["hops"], thr)
        sizes = np.array([col.plan(store, rng.integers(0, len(store), B)) for _ in range(32)])
        n_max, e_max = int(sizes[:, 0].max() * 1.03) + 64, int(sizes[:, 1].max() * 1.03) + 256
        nr, er, gr = n_max, e_max, B + bench.PAD_MOLS
        layout, nbytes = col.blob_layout(nr, er, gr, cfg["tasks"])
        for pinned in ((False, True) if torch.cuda.is_available() else (False,)):
            blob = torch.empty(nbytes, dtype=torch.uint8, pin_memory=pinned)
            ptr = [blob.data_ptr() + o for o, _, _ in layout]
            T = {"plan": 0.0, "write": 0.0, "csr": 0.0}
            for r in range(a.reps + 3):
                idx = rng.integers(0, len(store), B)
                t0 = time.perf_counter()
                col.plan(store, idx)
                t1 = time.perf_counter()
                col.write(ptr[:4], ptr[4], ptr[5], ptr[6], ptr[7], None, nr, er, bench.PAD_MOLS)
                t2 = time.perf_counter()
                feed._check(col._lib.aimx_collate_csr(col._h, ptr[4], er, ptr[5], nr, gr, cfg["hops"], *ptr[8:14]),
                            "csr")
                t3 = time.perf_counter()
                if r >= 3:
                    T["plan"] += t1 - t0
                    T["write"] += t2 - t1
                    T["csr"] += t3 - t2
            print(json.dumps({"config": a.config, "threads": thr, "pinned": pinned, "MB": round(nbytes / 1e6, 2),
                              **{k: round(v / a.reps * 1e3, 3) for k, v in T.items()}}), flush=True)


if __name__ == "__main__":
    main()
