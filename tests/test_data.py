"""Product batch construction (aimx.data) vs the reference's BFS + collate fixtures: bit-exact."""
import numpy as np

from conftest import load_golden
from aimx import data as adata
from aimx.synth import QM9Asset


def test_bfs_collate_qm9_bit_exact():
    z = load_golden("edges")
    mols = QM9Asset().molecules(range(64))
    for hops in (3, 4, 6):
        col = adata.collate(mols, hops)
        assert np.array_equal(col["edges"], z[f"edges_h{hops}"].astype(np.int64))
        assert np.array_equal(col["batch"], z[f"batch_h{hops}"].astype(np.int64))


def test_bfs_synthetic_6hops_bit_exact():
    z = load_golden("edges")
    mols, off = [], 0
    for n, nb in zip(z["syn_n_atoms"], z["syn_n_bonds"]):
        mols.append((int(n), z["syn_bonds"][off:off + nb].astype(np.int64), np.zeros((n, 4), np.int64)))
        off += nb
    col = adata.collate(mols, 6)
    assert np.array_equal(col["edges"], z["syn_edges_h6"].astype(np.int64))


def test_collate_empty_and_single_atom():
    mols = [(1, np.zeros((0, 2), np.int64), np.zeros((1, 4), np.int64))] * 3
    col = adata.collate(mols, 3)
    assert col["edges"].shape == (0, 2)
    assert col["batch"].tolist() == [0, 1, 2]
