"""Generate tests/golden/stream_small.h5 (+ stream_small_expected.npz): a byte-level fixture of the
reference's HDF5 dataset format (features.py:381-431, 537-596) for the native stream reader.

Records are built in the reference's layout (compute_all's dict, features.py:318-334): int8 atom
feature columns, max_hops int32 [2, E_h] hop arrays from the pure-Python BFS restatement
(aimx.data.bfs_multi_hop, itself bit-exact against the reference's BFS, tests/test_data.py),
int32 atomic numbers, empty stereo lists. They are pickled by Python's own pickle.dumps as the
reference does and written with the HDF5 C library (aimx.h5.write_hdf5 -> libaimx_h5.so). The
record mix covers what the reader must handle: QM9 molecules and 40-atom synthetic ones, a float /
numpy float64 / numpy float32 target, int and numpy int64 charges, two pickled None records
(unparseable SMILES, features.py:551-553) and one record without 'precomputed' (skipped by
molecular.py:255-256).

The expected outputs are the reference collate (aimx.data.collate, molecular.py:339-458 restated)
of the valid records decoded back with pickle.loads — independent of the C++ decoder.

    python tests/golden/make_stream_fixture.py
"""
import os
import pickle
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

from aimx import data as adata  # noqa: E402
from aimx import h5  # noqa: E402
from aimx.synth import QM9Asset, synth_molecules  # noqa: E402

MAX_HOPS = 3


def record(n, bonds, feats, target, charge, smiles):
    hops = adata.bfs_multi_hop(n, bonds, MAX_HOPS)
    f = np.asarray(feats).reshape(n, -1)
    return {"smiles": smiles, "target": target, "precomputed": {
        "multi_hop_edges": hops,
        "atom_features": {k: f[:, i].astype(np.int8) for i, k in enumerate(adata.FEATURE_KEYS)},
        "chiral_tensors": [], "cis_bonds_tensors": [], "trans_bonds_tensors": [],
        "total_charge": charge, "atomic_numbers": (f[:, 0] + 1).astype(np.int32), "processed_smiles": smiles}}


def build():
    rng = np.random.default_rng(2024)
    mols = QM9Asset().molecules(range(40)) + synth_molecules(20, seed=11)
    recs = []
    for i, (n, bonds, feats) in enumerate(mols):
        t = float(rng.normal())
        target = t if i % 3 == 0 else (np.float64(t) if i % 3 == 1 else np.float32(t))
        charge = int(rng.integers(-1, 2)) if i % 2 else np.int64(rng.integers(-1, 2))
        recs.append(record(n, bonds, feats, target, charge, f"mol{i}"))
    recs.insert(5, None)
    recs.insert(17, {"smiles": "bad", "target": 0.0, "precomputed": None})
    recs.insert(33, None)
    return recs


def expected(recs):
    valid = [(i, pickle.loads(pickle.dumps(r))) for i, r in enumerate(recs)
             if r is not None and r.get("precomputed") is not None]
    mols, hops = [], []
    for _, r in valid:
        p = r["precomputed"]
        f = np.stack([p["atom_features"][k].astype(np.int64) for k in adata.FEATURE_KEYS], 1)
        mols.append((f.shape[0], None, f))
        hops.append(p["multi_hop_edges"])
    col = adata.collate(mols, MAX_HOPS, hops=hops)
    return {"positions": np.array([i for i, _ in valid], np.int64), "edges": col["edges"], "feats": col["feats"],
            "batch": col["batch"], "n_atoms": col["n_atoms"],
            "targets": np.array([float(r["target"]) for _, r in valid], np.float32),
            "total_charges": np.array([float(r["precomputed"]["total_charge"]) for _, r in valid], np.float32)}


if __name__ == "__main__":
    recs = build()
    h5.write_hdf5(os.path.join(HERE, "stream_small.h5"), recs, MAX_HOPS)
    np.savez_compressed(os.path.join(HERE, "stream_small_expected.npz"), **expected(recs))
    print(f"wrote stream_small.h5 ({len(recs)} records)")
