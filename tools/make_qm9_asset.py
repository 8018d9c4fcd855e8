"""Build aimnet-x2d_amd/data/qm9_val_graphs.npz from the reference's QM9 sample split.

Runs only in the development container (reads /root/reference/sample-data/qm9/sample-splits/val.csv,
header at val.csv:1). The output is a compact, committed data asset: per-molecule heavy+H atom
features and bond lists produced by the RDKit-free featuriser (aimx/smiles.py). QM9-shaped
synthetic batches on the GPU box are resampled from it.
"""
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aimnet-x2d_amd"))
from aimx.smiles import SmilesError, featurize  # noqa: E402

SRC = "/root/reference/sample-data/qm9/sample-splits/val.csv"


def main():
    rows = list(csv.reader(open(SRC)))
    header, rows = rows[0], rows[1:]
    n_atoms, feats, bonds_i, bonds_j, nbonds, targets, charges, smiles = [], [], [], [], [], [], [], []
    dropped = 0
    for r in rows:
        try:
            f = featurize(r[0])
        except SmilesError:  # compute_all returns None -> precompute_all_and_filter drops it
            dropped += 1
            continue
        adj = f["adj"]
        iu, ju = np.nonzero(np.triu(adj, 1))
        n_atoms.append(adj.shape[0])
        feats.append(np.stack([f["atom_type"], f["hydrogen_count"], f["degree"], f["hybridization"]], 1))
        bonds_i.append(iu.astype(np.int16))
        bonds_j.append(ju.astype(np.int16))
        nbonds.append(len(iu))
        targets.append([float(x) for x in r[1:]])
        charges.append(f["total_charge"])
        smiles.append(r[0])
    out = os.path.join(ROOT, "aimnet-x2d_amd", "data", "qm9_val_graphs.npz")
    np.savez_compressed(
        out,
        n_atoms=np.array(n_atoms, np.int32),
        atom_feats=np.concatenate(feats).astype(np.int8),
        n_bonds=np.array(nbonds, np.int32),
        bond_i=np.concatenate(bonds_i),
        bond_j=np.concatenate(bonds_j),
        targets=np.array(targets, np.float32),
        target_names=np.array(header[1:]),
        total_charge=np.array(charges, np.float32),
        smiles=np.array(smiles),
    )
    na = np.array(n_atoms)
    print(out, os.path.getsize(out), "mols", len(na), "mean atoms", na.mean(), "max", na.max(),
          "mean bonds", np.mean(nbonds), "dropped", dropped)


if __name__ == "__main__":
    main()
