"""Native batch builder (libaimx_host.so) vs the reference's BFS + collate fixtures and vs the
Python restatement aimx.data: bit-exact. CPU only (the library has no GPU code)."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from aimx import data as adata
from aimx import feed
from aimx.synth import QM9Asset, synth_molecules


@pytest.fixture(scope="module")
def asset():
    return QM9Asset()


def _golden_syn_mols(z):
    mols, off = [], 0
    for n, nb in zip(z["syn_n_atoms"], z["syn_n_bonds"]):
        mols.append((int(n), z["syn_bonds"][off:off + nb].astype(np.int32), np.zeros((n, 4), np.int64)))
        off += nb
    return mols


def test_library_identity():
    assert feed.load_host().aimx_host_version().decode().startswith("aimx_host/")


def test_bfs_matches_python_restatement(asset):
    mols = asset.molecules(range(200)) + synth_molecules(50, seed=3)
    for n, bonds, _ in mols:
        for hops in (1, 3, 6):
            a = feed.bfs_multi_hop(n, bonds, hops)
            b = adata.bfs_multi_hop(n, bonds, hops)
            assert len(a) == len(b) == hops
            for x, y in zip(a, b):
                assert np.array_equal(x, y)


def test_bfs_duplicates_self_loops_and_empty():
    # duplicate bonds in both orientations and a self-loop collapse like `adj_matrix > 0`
    bonds = np.array([[0, 1], [1, 0], [1, 2], [2, 2], [0, 1]], np.int32)
    a = feed.bfs_multi_hop(3, bonds, 3)
    b = adata.bfs_multi_hop(3, bonds, 3)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert [h.shape[1] for h in a] == [4, 2, 0]
    assert [h.shape[1] for h in feed.bfs_multi_hop(1, np.zeros((0, 2), np.int32), 3)] == [0, 0, 0]
    with pytest.raises(feed.HostError):
        feed.bfs_multi_hop(2, np.array([[0, 2]], np.int32), 3)


@pytest.mark.parametrize("precompute", [0, 6])
@pytest.mark.parametrize("threads", [1, 3])
def test_collate_qm9_golden_bit_exact(asset, precompute, threads):
    z = load_golden("edges")
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=precompute, threads=threads)
    for hops in (3, 4, 6):
        col = feed.HostCollator(hops, threads).collate(store, np.arange(64))
        assert np.array_equal(col["edges"], z[f"edges_h{hops}"].astype(np.int64))
        assert np.array_equal(col["batch"], z[f"batch_h{hops}"].astype(np.int64))
        ref = adata.collate(asset.molecules(range(64)), hops)
        assert np.array_equal(col["feats"], ref["feats"])
        assert np.array_equal(col["n_atoms"], ref["n_atoms"])
        assert np.array_equal(col["total_charges"], asset.total_charge[:64])
        assert np.array_equal(col["targets"], asset.targets[:64])


def test_collate_synthetic_6hops_golden():
    z = load_golden("edges")
    store = feed.HostStore.from_molecules(_golden_syn_mols(z))
    col = feed.HostCollator(6, 2).collate(store, np.arange(len(z["syn_n_atoms"])))
    assert np.array_equal(col["edges"], z["syn_edges_h6"].astype(np.int64))


def test_collate_random_order_and_repeats(asset):
    rng = np.random.default_rng(7)
    idx = rng.integers(0, len(asset), 700)  # repeats allowed, as a sampler with replacement
    store = feed.HostStore.from_qm9_asset(asset, threads=4)
    col = feed.HostCollator(3, 4).collate(store, idx)
    ref = adata.collate(asset.molecules(idx), 3)
    for k in ("edges", "feats", "batch", "n_atoms"):
        assert np.array_equal(col[k], ref[k]), k


def test_collate_empty_and_single_atom():
    mols = [(1, np.zeros((0, 2), np.int32), np.zeros((1, 4), np.int64))] * 3
    store = feed.HostStore.from_molecules(mols)
    col = feed.HostCollator(3, 2).collate(store, np.arange(3))
    assert col["edges"].shape == (0, 2)
    assert col["batch"].tolist() == [0, 1, 2]
    col0 = feed.HostCollator(3, 2).collate(store, np.zeros(0, np.int64))
    assert col0["edges"].shape == (0, 2) and col0["batch"].shape == (0,)


def test_padding_matches_pad_collated(asset):
    idx = np.arange(100, 164)
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=3)
    c = feed.HostCollator(3, 3)
    n, e = c.plan(store, idx)
    n_max, e_max, pm = n + 37, e + 300, 8
    blob, layout, gr, nr, real = c.collate_blob(store, idx, pinned=False, n_max=n_max, e_max=e_max, pad_mols=pm)
    assert (gr, nr, real) == (64 + pm, n_max, (64, n, e))
    ref = adata.pad_collated(adata.collate(asset.molecules(idx), 3), n_max, e_max, 64, pm)
    b = adata.DeviceBatch.from_blob(blob, layout, gr, nr)
    assert np.array_equal(b.edges.numpy(), ref["edges"])
    assert np.array_equal(b.batch.numpy(), ref["batch"])
    for i, k in enumerate(adata.FEATURE_KEYS):
        assert np.array_equal(b.atom_features[k].numpy(), ref["feats"][:, i])
    tg = np.concatenate([asset.targets[idx], np.zeros((pm, 12), np.float32)])
    assert np.array_equal(b.targets.numpy(), tg)
    assert np.array_equal(b.total_charges.numpy()[:64], asset.total_charge[idx])
    with pytest.raises(feed.HostError):
        c.collate_blob(store, idx, pinned=False, n_max=n, e_max=e_max, pad_mols=pm)  # no padding atom


def test_blob_matches_device_batch_layout(asset):
    idx = np.arange(32)
    store = feed.HostStore.from_qm9_asset(asset)
    blob, layout, gr, nr, _ = feed.HostCollator(3, 2).collate_blob(store, idx, pinned=False)
    col = adata.collate(asset.molecules(idx), 3)
    ref = adata.DeviceBatch(col, "cpu", targets=asset.targets[idx], total_charges=asset.total_charge[idx])
    assert layout == ref._layout
    for o, dt, shape in layout:  # field bytes (alignment gaps are never read)
        nb = int(np.prod(shape)) * dt.itemsize
        assert torch.equal(blob[o:o + nb], ref._blob[o:o + nb])


def test_invalid_arguments(asset):
    store = feed.HostStore.from_qm9_asset(asset)
    c = feed.HostCollator(3, 2)
    with pytest.raises(feed.HostError):
        c.plan(store, np.array([len(asset)]))
    with pytest.raises(feed.HostError):
        c.plan(store, np.array([-1]))
    with pytest.raises(feed.HostError):  # bond index outside the molecule
        feed.HostStore([2], [np.array([[0, 5]])], np.zeros((2, 4), np.int32))
    with pytest.raises(feed.HostError):  # cache shorter than the collator's hops
        feed.HostCollator(4, 1).plan(feed.HostStore.from_qm9_asset(asset, precompute_hops=3), np.arange(4))


def test_host_library_exports_every_header_symbol_and_struct_layout():
    import os
    import re

    from conftest import ROOT
    src = open(os.path.join(ROOT, "include", "aimx_host.h")).read()
    syms = sorted(set(re.findall(r"^\s*(?:int|int64_t|void|const char\*)\s+(aimx_\w+)\s*\(", src, re.M)))
    assert len(syms) >= 10
    lib = feed.load_host()
    for s in syms:
        assert hasattr(lib, s), s
    body = re.search(r"typedef struct AimxCollateOut \{(.*?)\} AimxCollateOut;", src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"\**\s*(\w+)\s*(?:\[[^\]]*\])?\s*[;,]", body)
    assert names == [f[0] for f in feed.CollateOut._fields_]
