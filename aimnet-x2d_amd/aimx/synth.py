"""Synthetic molecular graphs for the c4/c5 configurations and for benches.

* 40-atom class: random heavy-atom tree (n_heavy ~ N(18, 2)), max valence drawn from {4,4,4,3,2},
  one ring closure per 6 heavy atoms, saturated with hydrogens appended after the heavy atoms
  (RDKit AddHs order, as the reference's featuriser produces, src/datasets/features.py:166-178).
* QM9 class: molecules resampled from the committed QM9-val graph asset (data/qm9_val_graphs.npz,
  produced by tools/make_qm9_asset.py from the reference's sample split).

Molecules are returned as (n_atoms, bonds int32 [B,2] (i<j), feats int64 [n,4]) with feature
columns (atom_type, hydrogen_count, degree, hybridization).
"""
from __future__ import annotations

import os

import numpy as np

_ASSET = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "qm9_val_graphs.npz")


def synth_molecule(rng, mean_heavy=18.0, sd_heavy=2.0):
    n = max(2, int(round(rng.normal(mean_heavy, sd_heavy))))
    val = rng.choice(np.array([4, 4, 4, 3, 2]), size=n)
    deg = np.zeros(n, np.int64)
    bonds = []
    adj = set()
    for i in range(1, n):
        cand = [j for j in range(i) if deg[j] < val[j]]
        if not cand:
            cand = list(range(i))
        j = int(cand[rng.integers(len(cand))])
        bonds.append((j, i))
        adj.add((j, i))
        deg[i] += 1
        deg[j] += 1
    for _ in range(n // 6):
        free = [k for k in range(n) if deg[k] < val[k]]
        if len(free) < 2:
            break
        for _try in range(8):
            a, b = rng.choice(free, 2, replace=False)
            a, b = int(min(a, b)), int(max(a, b))
            if (a, b) not in adj:
                bonds.append((a, b))
                adj.add((a, b))
                deg[a] += 1
                deg[b] += 1
                break
    nh = np.maximum(val - deg, 0)
    total = n + int(nh.sum())
    nxt = n
    for k in range(n):
        for _ in range(int(nh[k])):
            bonds.append((k, nxt))
            nxt += 1
    feats = np.stack([
        rng.integers(0, 119, total), rng.integers(0, 9, total),
        rng.integers(0, 7, total), rng.integers(0, 7, total)], 1).astype(np.int64)
    return total, np.array(bonds, np.int32).reshape(-1, 2), feats


def synth_molecules(count, seed=0):
    rng = np.random.default_rng(seed)
    return [synth_molecule(rng) for _ in range(count)]


class QM9Asset:
    """Committed QM9-val graphs (13,373 molecules, 17.9 atoms incl. H on average; the 16 SMILES RDKit would reject are dropped)."""

    def __init__(self, path=_ASSET):
        z = np.load(path, allow_pickle=False)
        self.n_atoms = z["n_atoms"].astype(np.int64)
        self.n_bonds = z["n_bonds"].astype(np.int64)
        self.atom_off = np.concatenate([[0], np.cumsum(self.n_atoms)])
        self.bond_off = np.concatenate([[0], np.cumsum(self.n_bonds)])
        self.feats = z["atom_feats"].astype(np.int64)
        self.bi = z["bond_i"].astype(np.int32)
        self.bj = z["bond_j"].astype(np.int32)
        self.targets = z["targets"]
        self.total_charge = z["total_charge"]
        self.smiles = z["smiles"]

    def __len__(self):
        return len(self.n_atoms)

    def molecule(self, i):
        a0, a1 = self.atom_off[i], self.atom_off[i + 1]
        b0, b1 = self.bond_off[i], self.bond_off[i + 1]
        bonds = np.stack([self.bi[b0:b1], self.bj[b0:b1]], 1)
        return int(self.n_atoms[i]), bonds, self.feats[a0:a1]

    def molecules(self, idx):
        return [self.molecule(int(i)) for i in idx]


def adjacency(n, bonds):
    adj = np.zeros((n, n), np.int32)
    if len(bonds):
        adj[bonds[:, 0], bonds[:, 1]] = 1
        adj[bonds[:, 1], bonds[:, 0]] = 1
    return adj
