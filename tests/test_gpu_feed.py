"""GPU: the native batch feed (C++ collate -> pinned blob -> async H2D on a copy stream) delivers
batches bit-identical to the Python-built DeviceBatch, in order, and the model step consumes them
(the GNN forward on a fed batch equals the forward on the Python-built batch bit for bit)."""
import numpy as np
import pytest
import torch

from aimx import data as adata
from aimx import feed
from aimx.synth import QM9Asset

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import aimx
    aimx.load()


def _fields(b):
    c = b.edges._aimx_csr
    return [b.edges, b.batch, b.total_charges, b.targets] + [b.atom_features[k] for k in adata.FEATURE_KEYS] + \
        [c.fwd_rowptr, c.fwd_col, c.bwd_rowptr, c.bwd_col, c.graph_rowptr, c.graph_col]


@pytest.mark.parametrize("pad,ring", [(False, False), (True, False), (True, True)])
def test_feeder_batches_bit_exact_and_ordered(pad, ring):
    asset = QM9Asset()
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=3, threads=3)
    rng = np.random.default_rng(11)
    idxs = [rng.integers(0, len(asset), 96) for _ in range(7)]
    n_max = e_max = pm = 0
    if pad:
        c = feed.HostCollator(3, 1)
        sizes = np.array([c.plan(store, i) for i in idxs])
        n_max, e_max, pm = int(sizes[:, 0].max()) + 5, int(sizes[:, 1].max()) + 9, 8
    f = feed.BatchFeeder(store, iter(idxs), 3, DEV, depth=2, threads=3, n_max=n_max, e_max=e_max, pad_mols=pm,
                         ring=ring)
    got = list(f)
    assert len(got) == len(idxs)
    for b, idx in zip(got, idxs):
        col = adata.collate(asset.molecules(idx), 3)
        tg, tc = asset.targets[idx], asset.total_charge[idx]
        if pad:
            col = adata.pad_collated(col, n_max, e_max, len(idx), pm)
            tg = np.concatenate([tg, np.zeros((pm, tg.shape[1]), np.float32)])
            tc = np.concatenate([tc, np.zeros(pm, np.float32)])
        ref = adata.DeviceBatch(col, DEV, targets=tg, total_charges=tc, csr_hops=3)
        assert b._layout == ref._layout
        for x, y in zip(_fields(b), _fields(ref)):
            assert torch.equal(x, y)
        assert b.real_graphs == len(idx)


def test_fed_batch_drives_model_identically():
    from models import GNN
    asset = QM9Asset()
    store = feed.HostStore.from_qm9_asset(asset, threads=2)  # BFS per batch (streaming mode)
    idx = np.arange(200, 264)
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    torch.manual_seed(0)
    m = GNN(fs, 128, 1, num_shells=3).to(DEV).eval()
    b = next(iter(feed.BatchFeeder(store, iter([idx]), 3, DEV, depth=1, threads=2)))
    ref = adata.DeviceBatch(adata.collate(asset.molecules(idx), 3), DEV, targets=asset.targets[idx],
                            total_charges=asset.total_charge[idx])
    from aimx.plan import GraphPlan
    assert GraphPlan(b.num_atoms, 3, edges=b.edges, batch=b.batch, num_graphs=b.num_graphs).host_csr
    assert not GraphPlan(ref.num_atoms, 3, edges=ref.edges, batch=ref.batch, num_graphs=ref.num_graphs).host_csr
    with torch.no_grad():
        o1 = m(*b.model_args())[0]  # CSR views built by the batch builder
        o2 = m(*ref.model_args())[0]  # CSR views built on the device
    assert torch.equal(o1, o2)


def test_feeder_surfaces_collate_errors():
    asset = QM9Asset()
    store = feed.HostStore.from_qm9_asset(asset)
    f = feed.BatchFeeder(store, iter([np.array([0, len(asset)])]), 3, DEV, depth=1)
    with pytest.raises(feed.HostError):
        next(f)


def test_feeder_ring_reuse_is_race_free():
    """Static shapes: the ring reuses a slot only after the consumer has moved past its batch. A
    busy consumer stream (long GEMMs queued before each batch is read) lets the copy stream run
    ahead; every batch read must still equal the host-collated blob byte for byte. Consumed one at
    a time the ring stays a few slots; kept (list) it grows instead of overwriting."""
    asset = QM9Asset()
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=3, threads=3)
    rng = np.random.default_rng(5)
    idxs = [rng.integers(0, len(asset), 64) for _ in range(24)]
    c = feed.HostCollator(3, 2)
    sizes = np.array([c.plan(store, i) for i in idxs])
    pad = (int(sizes[:, 0].max()) + 7, int(sizes[:, 1].max()) + 11, 4)
    want = [c.collate_blob(store, i, False, *pad)[0].clone() for i in idxs]
    layout = c.collate_blob(store, idxs[0], False, *pad)[1]

    def same(a, b):  # every field's bytes (the 256-byte alignment gaps are never written)
        return all(torch.equal(a[o:o + int(np.prod(sh)) * np.dtype(dt).itemsize],
                               b[o:o + int(np.prod(sh)) * np.dtype(dt).itemsize]) for o, dt, sh in layout)
    f = feed.BatchFeeder(store, iter(idxs), 3, DEV, depth=2, threads=2, n_max=pad[0], e_max=pad[1], pad_mols=pad[2],
                         ring=True)
    x = torch.randn(2048, 2048, device=DEV)
    got = []
    for b in f:
        for _ in range(4):
            x = torch.tanh(x @ x)
        got.append(b._blob.clone())
    torch.cuda.synchronize()
    assert len(got) == len(idxs)
    for g, w in zip(got, want):
        assert same(g.cpu(), w)
    assert f.stats()["ring"] <= 6
    kept = list(feed.BatchFeeder(store, iter(idxs), 3, DEV, depth=2, threads=2, n_max=pad[0], e_max=pad[1],
                                 pad_mols=pad[2], ring=True))
    torch.cuda.synchronize()
    for b, w in zip(kept, want):
        assert same(b._blob.cpu(), w)


@pytest.mark.parametrize("ring", [False, True])
def test_overflow_batch_goes_out_unpadded(ring):
    """Static shapes from a few sample batches: a later batch above that capacity is handed out
    unpadded (its own layout, bit-exact to the dynamic collate) and counted, the others padded."""
    asset = QM9Asset()
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=3, threads=2)
    rng = np.random.default_rng(2)
    idxs = [rng.integers(0, len(asset), 64) for _ in range(10)]
    c = feed.HostCollator(3, 2)
    sizes = np.array([c.plan(store, i) for i in idxs])
    big = int(np.argmax(sizes[:, 1]))
    rest = [k for k in range(len(idxs)) if k != big]
    n_max, e_max = int(sizes[rest, 0].max()) + 3, int(sizes[rest, 1].max())
    assert sizes[big, 1] > e_max
    f = feed.BatchFeeder(store, iter(idxs), 3, DEV, depth=2, threads=2, n_max=n_max, e_max=e_max, pad_mols=6,
                         ring=ring)
    got = [b for b in f]
    torch.cuda.synchronize()
    assert f.stats()["overflow"] == 1
    for k, (b, idx) in enumerate(zip(got, idxs)):
        col = adata.collate(asset.molecules(idx), 3)
        tg, tc = asset.targets[idx], asset.total_charge[idx]
        if k != big:
            col = adata.pad_collated(col, n_max, e_max, len(idx), 6)
            tg = np.concatenate([tg, np.zeros((6, tg.shape[1]), np.float32)])
            tc = np.concatenate([tc, np.zeros(6, np.float32)])
        ref = adata.DeviceBatch(col, DEV, targets=tg, total_charges=tc, csr_hops=3)
        assert b._layout == ref._layout, k
        for x, y in zip(_fields(b), _fields(ref)):
            assert torch.equal(x, y)
        assert b.real_graphs == len(idx)


def test_kept_views_stay_valid_without_ring():
    """The default feeder (ring=False) gives every static-shape batch a blob of its own: a consumer
    that keeps only tensor views (batch.targets for an epoch metric, batch.batch), never the batch
    object, still reads each batch's own values after the feeder has moved on, with a busy stream."""
    asset = QM9Asset()
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=3, threads=2)
    rng = np.random.default_rng(9)
    idxs = [rng.integers(0, len(asset), 64) for _ in range(16)]
    c = feed.HostCollator(3, 2)
    sizes = np.array([c.plan(store, i) for i in idxs])
    pad = (int(sizes[:, 0].max()) + 7, int(sizes[:, 1].max()) + 11, 4)
    f = feed.BatchFeeder(store, iter(idxs), 3, DEV, depth=2, threads=2, n_max=pad[0], e_max=pad[1], pad_mols=pad[2])
    x = torch.randn(1024, 1024, device=DEV)
    targets, mols = [], []
    for b in f:
        x = torch.tanh(x @ x)
        targets.append(b.targets[:b.real_graphs])
        mols.append(b.batch)
        del b
    torch.cuda.synchronize()
    for t, m, idx in zip(targets, mols, idxs):
        assert torch.equal(t.cpu(), torch.from_numpy(asset.targets[idx]))
        assert torch.equal(m[:len(m) - (m >= len(idx)).sum()].cpu(),
                           torch.from_numpy(adata.collate(asset.molecules(idx), 3)["batch"]))
