"""GPU: the drop-in autograph (aimx/autograph.py). An unchanged eager training loop
(reference trainer.py:151-164) with AIMX_AUTOGRAPH on must give the eager path's outputs,
gradients and parameter trajectory; the padding of its shape buckets must not leak into any real
molecule."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = dict(source="qm9", hidden=128, hops=3, batch=64, tasks=1, pc=False)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import aimx
    aimx.load()


def _model(seed=0, dropout=0.0, pc=False, ag=False):
    """ag: the autograph on (the default for GNN) or off (every operator launched eagerly)."""
    from aimx import autograph
    from models import GNN
    torch.manual_seed(seed)
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, CFG["hidden"], 1, num_shells=3, dropout=dropout, shell_conv_dropout=dropout, ffn_dropout=dropout,
            use_partial_charges=pc).to(DEV).train()
    return autograph.enable(m, ag)


def _batches(n, seed, batch=None):
    import bench
    cfg = dict(CFG, batch=batch or CFG["batch"])
    return bench.make_batches(cfg, n, seed, DEV, pad=False)


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("pc", [False, True])
def test_autograph_matches_eager_forward_and_gradients(pc):
    from aimx import autograph
    b = _batches(1, 11)[0]
    m1 = _model(pc=pc)
    m2 = _model(pc=pc)
    m2.load_state_dict(m1.state_dict())
    autograph.enable(m2)
    for _ in range(2):  # first call captures the bucket, second replays it
        for m in (m1, m2):
            m.zero_grad(set_to_none=True)
        o1, a1, q1 = m1(*b.model_args())
        o2, a2, q2 = m2(*b.model_args())
        (o1.square().sum() + o1.sum()).backward()
        (o2.square().sum() + o2.sum()).backward()
        assert o2.shape == o1.shape and _rel(o2, o1) < 1e-6
        assert a2.shape == a1.shape and _rel(a2, a1) < 1e-6
        if pc:
            assert q2.shape == q1.shape and _rel(q2, q1) < 1e-6
        for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
            if p1.grad is None:
                assert p2.grad is None, k
                continue
            assert _rel(p2.grad, p1.grad) < 1e-5, k
    st = m2.__dict__["_aimx_autograph_state"]
    assert len(st.buckets) == 1


def test_capture_leaves_no_stale_accumulate_grad_nodes():
    """The capture's warm-up graph must be gone before the capture: alive, it would hand the
    captured backward the warm-up stream's AccumulateGrad nodes (torch's stream-mismatch warning,
    extra synchronisation)."""
    import warnings
    from aimx import autograph
    from aimx.train import GraphedTrainStep
    from aimx.optim import FusedAdam
    from models import L1Loss
    b = _batches(1, 12)[0]
    m = autograph.enable(_model(), True)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for _ in range(3):
            m.zero_grad(set_to_none=True)
            out, _, _ = m(*b.model_args())
            out.sum().backward()
        m2 = _model()
        step = GraphedTrainStep(m2, L1Loss(), FusedAdam(m2.parameters(), lr=1e-3), b)
        for _ in range(2):
            step(b)
        torch.cuda.synchronize()
    bad = [str(x.message) for x in w if "AccumulateGrad" in str(x.message)]
    assert not bad, bad[0]


def test_autograph_training_tracks_eager_over_buckets():
    """Adam over batches of two sizes (two shape buckets, each replayed): same trajectory."""
    from aimx import autograph
    from aimx.optim import FusedAdam
    from models import L1Loss
    bs = _batches(3, 21) + _batches(2, 22, batch=40)
    order = [0, 3, 1, 4, 2, 0, 3]
    m1 = _model()
    m2 = _model()
    m2.load_state_dict(m1.state_dict())
    autograph.enable(m2)
    o1 = FusedAdam(m1.parameters(), lr=1e-3, max_grad_norm=1.0)
    o2 = FusedAdam(m2.parameters(), lr=1e-3, max_grad_norm=1.0)
    crit = L1Loss()
    l1s, l2s = [], []
    for i in order:
        b = bs[i]
        for m, o, ls in ((m1, o1, l1s), (m2, o2, l2s)):
            o.zero_grad(set_to_none=True)
            out, _, _ = m(*b.model_args())
            loss = crit(out, b.targets)
            loss.backward()
            o.step()
            ls.append(loss.item())
    np.testing.assert_allclose(l2s, l1s, rtol=1e-4, atol=1e-6)
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert (p1 - p2).abs().max().item() <= 1e-4 * max(1.0, p1.abs().max().item()), k
    assert len(m2.__dict__["_aimx_autograph_state"].buckets) == 2


def test_autograph_accumulates_without_set_to_none():
    from aimx import autograph
    b = _batches(1, 31)[0]
    m1 = _model()
    m2 = _model()
    m2.load_state_dict(m1.state_dict())
    autograph.enable(m2)
    for m in (m1, m2):
        for _ in range(2):  # two backward passes into the same .grad (gradient accumulation)
            out, _, _ = m(*b.model_args())
            out.sum().backward()
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        if p1.grad is not None:
            assert _rel(p2.grad, p1.grad) < 1e-5, k
    for m in (m1, m2):
        m.zero_grad(set_to_none=False)  # in-place zero: the next backward must not add stale values
        out, _, _ = m(*b.model_args())
        out.sum().backward()
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        if p1.grad is not None:
            assert _rel(p2.grad, p1.grad) < 1e-5, k


def test_autograph_is_the_default_and_reuses_buckets():
    """GNN's training forward goes through the autograph unless AIMX_AUTOGRAPH=0; batches that fit a
    live bucket (same molecule count) reuse it instead of capturing another."""
    import os
    from aimx import autograph
    from models import GNN
    assert os.environ.get("AIMX_AUTOGRAPH", "1") != "0"
    torch.manual_seed(0)
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, CFG["hidden"], 1, num_shells=3).to(DEV).train()
    bs = sorted(_batches(4, 51), key=lambda b: -b.num_atoms)
    for b in bs:
        assert autograph.wanted(m, b.model_args())
        out, _, _ = m(*b.model_args())
        out.sum().backward()
        m.zero_grad(set_to_none=True)
    assert len(m.__dict__["_aimx_autograph_state"].buckets) == 1


def test_autograph_falls_back_and_guards():
    from aimx import autograph
    from aimx._lib import AimxError
    b = _batches(1, 41)[0]
    m = _model()
    autograph.enable(m)
    with torch.no_grad():
        m(*b.model_args())  # grad disabled: eager, no bucket
    m.eval()
    m(*b.model_args())      # eval mode: eager
    m.train()
    assert not m.__dict__.get("_aimx_autograph_state") or not m.__dict__["_aimx_autograph_state"].buckets
    o1, _, _ = m(*b.model_args())
    o2, _, _ = m(*b.model_args())  # second forward of the same bucket before the first backward
    o2.sum().backward()
    with pytest.raises(AimxError):
        o1.sum().backward()
    h = m.pooling.register_forward_hook(lambda *a: None)
    try:
        assert not autograph.wanted(m, b.model_args())  # module hooks would stop firing on replay
    finally:
        h.remove()


def test_autograph_size_gate(monkeypatch):
    """By default the replay applies only while atoms x hidden <= MAX_WORK (device-bound larger steps
    run eagerly: measured faster at c4 / c5); enable(model, True) forces it."""
    from aimx import autograph
    from models import GNN
    b = _batches(1, 71)[0]
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, CFG["hidden"], 1, num_shells=3).to(DEV).train()
    assert autograph.wanted(m, b.model_args())
    monkeypatch.setattr(autograph, "MAX_WORK", b.num_atoms * CFG["hidden"] - 1)
    assert not autograph.wanted(m, b.model_args())
    autograph.enable(m, True)
    assert autograph.wanted(m, b.model_args())


def test_autograph_amp_state_and_replaced_parameters():
    """The autocast state is part of the bucket key (a capture bakes in bf16 or fp32 GEMM operands):
    the same batch under autocast gets its own bucket and matches the eager AMP path; replacing the
    Parameter objects (load_state_dict(assign=True)) re-captures instead of replaying stale weights."""
    from aimx import autograph
    b = _batches(1, 61)[0]
    m1 = _model()
    m2 = _model()
    m2.load_state_dict(m1.state_dict())
    autograph.enable(m2)
    for amp in (False, True, False, True):
        outs = []
        for m in (m1, m2):
            m.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                out, _, _ = m(*b.model_args())
            out.sum().backward()
            outs.append(out.detach())
        assert _rel(outs[1], outs[0]) < 1e-5, amp
    st = m2.__dict__["_aimx_autograph_state"]
    assert len(st.buckets) == 2
    with torch.no_grad():  # new Parameter objects with new values
        sd = {k: v * 1.5 for k, v in m1.state_dict().items()}
    m1.load_state_dict(sd)
    m2.load_state_dict(sd, assign=True)
    o1 = m1(*b.model_args())[0]
    o2 = m2(*b.model_args())[0]
    assert _rel(o2.detach(), o1.detach()) < 1e-5
    o2.sum().backward()
    assert all(p.grad is not None for n, p in m2.named_parameters() if "long_range" not in n)


def test_autograph_recaptures_after_storage_swap():
    """`p.data = ...` on the same Parameter objects (torch.nn.utils.vector_to_parameters, EMA / SWA
    weight swaps) registers nothing, but moves the storage a captured graph reads: the next step
    must re-capture, not replay stale (possibly freed) parameter memory."""
    from torch.nn.utils import parameters_to_vector, vector_to_parameters
    from aimx import autograph
    b = _batches(1, 67)[0]
    m1 = _model()
    m2 = _model()
    m2.load_state_dict(m1.state_dict())
    autograph.enable(m2)
    for _ in range(2):  # capture, then replay
        m2.zero_grad(set_to_none=True)
        m2(*b.model_args())[0].sum().backward()
    st = m2.__dict__["_aimx_autograph_state"]
    old = list(st.buckets.values())  # held: a freed bucket's id() could be reused by its successor
    with torch.no_grad():
        vec = parameters_to_vector(m2.parameters()) * 1.25
        vector_to_parameters(vec, m2.parameters())
        m1.load_state_dict({k: v * 1.25 for k, v in m1.state_dict().items()})
    for m in (m1, m2):
        m.zero_grad(set_to_none=True)
    o1 = m1(*b.model_args())[0]
    o2 = m2(*b.model_args())[0]
    assert not any(bk is o for bk in st.buckets.values() for o in old)  # the bucket was re-captured
    assert _rel(o2.detach(), o1.detach()) < 1e-5
    o1.sum().backward()
    o2.sum().backward()
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        if p1.grad is not None:  # absolute floor: the pool's softmax-logit bias has an exactly-zero gradient
            assert (p2.grad - p1.grad).norm().item() <= 1e-5 * max(p1.grad.norm().item(), 1e-9), n


@pytest.mark.parametrize("slack", [1, 7, 8, 9, 300])
def test_pad_batch_matches_pad_collated(slack):
    """aimx_pad_batch (one launch) builds exactly aimx.data.pad_collated's static layout: real rows
    copied, slack atoms in 8 near-equal padding molecules, slack edges self-pairs over them."""
    import ctypes
    from aimx import _lib
    from aimx.autograph import PAD_MOLS
    from aimx.data import FEATURE_KEYS, pad_collated
    from aimx._lib import check, ptr, stream_ptr
    b = _batches(1, 61)[0]
    N, E, G = b.num_atoms, b.edges.shape[0], b.num_graphs
    Np, Ep = N + slack, E + 3 * slack + 5
    col = {"feats": np.stack([b.atom_features[k].cpu().numpy() for k in FEATURE_KEYS], 1),
           "edges": b.edges.cpu().numpy(), "batch": b.batch.cpu().numpy(), "n_atoms": np.zeros(G, np.int64)}
    ref = pad_collated(col, Np, Ep, G, PAD_MOLS)
    feat = torch.full((4, Np), -1, dtype=torch.int64, device=DEV)
    edges = torch.full((Ep, 2), -1, dtype=torch.int64, device=DEV)
    batch = torch.full((Np,), -1, dtype=torch.int64, device=DEV)
    charges = torch.full((G + PAD_MOLS,), -1.0, device=DEV)
    a = _lib.PadBatch()
    for i, k in enumerate(FEATURE_KEYS):
        a.feat[i], a.feat_stride[i] = b.atom_features[k].data_ptr(), b.atom_features[k].stride(0)
    a.edges, a.edge_s0, a.edge_s1 = b.edges.data_ptr(), b.edges.stride(0), b.edges.stride(1)
    a.batch, a.batch_stride = b.batch.data_ptr(), b.batch.stride(0)
    a.charges, a.charge_stride = b.total_charges.data_ptr(), b.total_charges.stride(0)
    a.N, a.E, a.G = N, E, G
    a.out_feat, a.out_edges, a.out_batch, a.out_charges = ptr(feat), ptr(edges), ptr(batch), ptr(charges)
    a.Np, a.Ep, a.pad_mols = Np, Ep, PAD_MOLS
    check(_lib.load().aimx_pad_batch(ctypes.byref(a), stream_ptr(b.edges.device)), "pad_batch")
    torch.cuda.synchronize()
    assert np.array_equal(feat.cpu().numpy().T, ref["feats"])
    assert np.array_equal(edges.cpu().numpy(), ref["edges"])
    assert np.array_equal(batch.cpu().numpy(), ref["batch"])
    q = charges.cpu().numpy()
    assert np.array_equal(q[:G], b.total_charges.cpu().numpy()) and not q[G:].any()
    a.Np = N  # no slack atom: rejected
    assert _lib.load().aimx_pad_batch(ctypes.byref(a), stream_ptr(b.edges.device)) != 0


def test_autograph_grad_hooks_fire_through_autograd():
    """Gradient hooks on the parameters (what DDP's reducer relies on): the replay hands its
    gradients out through autograd (_ReplayGrads), so every used parameter's post-accumulate hook
    fires once per backward with the replayed gradient, equal to the eager gradients; the unused
    long_range_projection gets none, as eagerly."""
    from aimx import autograph
    b = _batches(1, 13)[0]
    m1 = _model()
    m2 = _model()
    m2.load_state_dict(m1.state_dict())
    autograph.enable(m2)
    seen = {}
    hs = [p.register_post_accumulate_grad_hook(lambda p, n=n: seen.__setitem__(n, seen.get(n, 0) + 1))
          for n, p in m2.named_parameters()]
    try:
        for it in range(2):
            for m in (m1, m2):
                m.zero_grad(set_to_none=True)
            o1, _, _ = m1(*b.model_args())
            o2, _, _ = m2(*b.model_args())
            (o1.square().sum() + o1.sum()).backward()
            (o2.square().sum() + o2.sum()).backward()
            torch.cuda.synchronize()
            assert autograph._state(m2).buckets, "the replay did not run"
            used = {n for n, p in m1.named_parameters() if p.grad is not None}
            assert set(seen) == used and all(v == it + 1 for v in seen.values()), seen
            for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
                if p1.grad is None:
                    assert p2.grad is None, n
                else:
                    assert _rel(p2.grad, p1.grad) < 1e-5, n
    finally:
        for h in hs:
            h.remove()


def test_autograph_hooked_accumulation_without_zero_grad():
    """through autograd (_ReplayGrads, here via a post-accumulate hook) the first
    backward hands out fresh views of the bucket's static gradients. A second forward/backward
    WITHOUT zero_grad (gradient accumulation, DDP no_sync micro-batches) replays into that same
    memory: each .grad must end as g_old + g_new (eager), not 2 g_new. Two batches of the same
    bucket, then a third step after zero_grad(set_to_none=False)."""
    from aimx import autograph
    bs = _batches(2, 17)
    m1 = _model()
    m2 = _model()
    m2.load_state_dict(m1.state_dict())
    autograph.enable(m2)
    hs = [p.register_post_accumulate_grad_hook(lambda p: None) for p in m2.parameters()]
    try:
        for m in (m1, m2):
            m.zero_grad(set_to_none=True)
        for k, b in enumerate(bs + [bs[0]]):
            if k == 2:
                for m in (m1, m2):
                    m.zero_grad(set_to_none=False)
            for m in (m1, m2):
                o, _, _ = m(*b.model_args())
                (o.square().sum() + o.sum()).backward()
            torch.cuda.synchronize()
            assert autograph._state(m2).buckets, "the replay did not run"
            for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
                if p1.grad is None:
                    assert p2.grad is None, n
                else:
                    assert _rel(p2.grad, p1.grad) < 1e-5, (k, n, _rel(p2.grad, p1.grad))
    finally:
        for h in hs:
            h.remove()
