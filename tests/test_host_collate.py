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
    ref = adata.DeviceBatch(col, "cpu", targets=asset.targets[idx], total_charges=asset.total_charge[idx], csr_hops=3)
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


# ------------------------------------------------------------------------------- host CSR views
def _oracle_graph():
    import importlib
    return importlib.import_module("oracle.graph")


@pytest.mark.parametrize("case,h", [("c1", 3), ("c2", 3), ("c3", 4), ("c5s", 6)])
def test_host_csr_matches_oracle_stable_sort(case, h):
    """aimx_csr_host_build == the oracle's stable CSR (the reference's scatter order) on the
    golden batches, for all three views; and the DeviceBatch carries them on its edges tensor."""
    og = _oracle_graph()
    z = load_golden(case)
    e = z["edges"].astype(np.int64)
    b = z["batch"].astype(np.int64)
    n, g = b.shape[0], len(z["n_mol_atoms"])
    col = {"edges": e, "feats": z["feats"].astype(np.int64), "batch": b, "n_atoms": z["n_mol_atoms"]}
    db = adata.DeviceBatch(col, "cpu", csr_hops=h)
    hc = db.edges._aimx_csr
    assert (hc.hops, hc.N, hc.E, hc.G) == (h, n, e.shape[0], g)
    for (rp, cl), (keys, vals, rows) in zip(
            [(hc.fwd_rowptr, hc.fwd_col), (hc.bwd_rowptr, hc.bwd_col), (hc.graph_rowptr, hc.graph_col)],
            [(e[:, 0], np.mod(e[:, 1], n), h * n), (np.mod(e[:, 1], n), e[:, 0], n), (b, np.arange(n), g)]):
        rref, cref = og.stable_csr(keys, vals, rows)
        assert np.array_equal(rp.numpy(), rref)
        assert np.array_equal(cl.numpy(), cref)


def test_host_csr_general_contract_and_errors():
    """Hop-offset targets, negative and >= N sources (Python-style mod); out-of-range target or
    batch index -> HostError (the device builder's status word)."""
    og = _oracle_graph()
    rng = np.random.default_rng(5)
    n, h, e, g = 300, 4, 20000, 7
    t = rng.integers(0, h * n, e)
    s = rng.integers(-5 * n, 5 * n, e)
    edges = np.stack([t, s], 1).astype(np.int64)
    batch = np.sort(rng.integers(0, g, n)).astype(np.int64)
    views = [np.empty(h * n + 1, np.int32), np.empty(e, np.int32), np.empty(n + 1, np.int32), np.empty(e, np.int32),
             np.empty(g + 1, np.int32), np.empty(n, np.int32)]
    adata.host_csr_into(views, edges, batch, g, h)
    rp, col = og.stable_csr(t, np.mod(s, n), h * n)
    assert np.array_equal(views[0], rp) and np.array_equal(views[1], col)
    rp, col = og.stable_csr(np.mod(s, n), t, n)
    assert np.array_equal(views[2], rp) and np.array_equal(views[3], col)
    bad = edges.copy()
    bad[11, 0] = h * n
    with pytest.raises(feed.HostError):
        adata.host_csr_into(views, bad, batch, g, h)
    bb = batch.copy()
    bb[3] = g
    with pytest.raises(feed.HostError):
        adata.host_csr_into(views, edges, bb, g, h)
    # no edges: empty fwd/bwd rows, graph CSR still built
    adata.host_csr_into(views, np.zeros((0, 2), np.int64), batch, g, h)
    assert views[0][-1] == 0 and views[2][-1] == 0 and views[4][-1] == n


def test_feeder_blob_carries_host_csr(asset):
    idx = np.arange(40, 104)
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=3)
    c = feed.HostCollator(3, 2)
    n, e = c.plan(store, idx)
    blob, layout, gr, nr, _ = c.collate_blob(store, idx, pinned=False, n_max=n + 20, e_max=e + 50, pad_mols=8)
    b = adata.DeviceBatch.from_blob(blob, layout, gr, nr, 3)
    col = adata.pad_collated(adata.collate(asset.molecules(idx), 3), n + 20, e + 50, 64, 8)
    ref = adata.DeviceBatch(col, "cpu", targets=np.zeros((72, 12), np.float32), csr_hops=3)
    assert layout == ref._layout
    a, r = b.edges._aimx_csr, ref.edges._aimx_csr
    for k in ("fwd_rowptr", "fwd_col", "bwd_rowptr", "bwd_col", "graph_rowptr", "graph_col"):
        assert torch.equal(getattr(a, k), getattr(r, k)), k


def _csr_views(nr, er, gr, h):
    return [np.empty(h * nr + 1, np.int32), np.empty(er, np.int32), np.empty(nr + 1, np.int32),
            np.empty(er, np.int32), np.empty(gr + 1, np.int32), np.empty(nr, np.int32)]


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_collator_parallel_csr_equals_serial(asset, threads):
    """aimx_collate_csr (the collator's pool, rows per molecule) == aimx_csr_host_build (one
    global stable sort), padded and unpadded batches, repeats, 3 and 6 hops; a batch whose edges
    cross molecules (not the collator's shape) takes the serial build and still agrees."""
    lib = feed.load_host()
    rng = np.random.default_rng(threads)
    stores = [(feed.HostStore.from_qm9_asset(asset, precompute_hops=3), 3),
              (feed.HostStore.from_molecules(synth_molecules(300, seed=2), precompute_hops=6), 6)]
    for store, h in stores:
        c = feed.HostCollator(h, threads)
        for trial in range(4):
            idx = rng.integers(0, len(store), int(rng.integers(1, 90)))
            n, e = c.plan(store, idx)
            pad = trial % 2 == 1
            nr, er, gr = (n + 37, e + 101, len(idx) + 3) if pad else (n, e, len(idx))
            feats = [np.empty(nr, np.int64) for _ in range(4)]
            edges = np.empty((er, 2), np.int64)
            batch = np.empty(nr, np.int64)
            c.write([f.ctypes.data for f in feats], edges.ctypes.data, batch.ctypes.data, n_max=nr if pad else 0,
                    e_max=er if pad else 0, pad_mols=3 if pad else 0)
            for mutate in (False, True):
                if mutate and er > 1:  # one edge joins molecules 0 and the last: not the collator's shape
                    edges[0, 1] = nr - 1
                got, ref = _csr_views(nr, er, gr, h), _csr_views(nr, er, gr, h)
                feed._check(lib.aimx_collate_csr(c._h, edges.ctypes.data, er, batch.ctypes.data, nr, gr, h,
                                                 *[v.ctypes.data for v in got]), "collate_csr")
                adata.host_csr_into(ref, edges, batch, gr, h)
                for a, b in zip(got, ref):
                    assert np.array_equal(a, b)
