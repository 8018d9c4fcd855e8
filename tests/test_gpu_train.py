"""GPU: the train loop (aimx.train, reference trainer.py:102-183). The graphed step replays the
eager step's numerics on the same padded batches, and training on QM9 reduces the loss."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import aimx
    aimx.load()


def _setup(seed=0, dropout=0.0):
    from aimx import feed
    from aimx.optim import FusedAdam
    from aimx.synth import QM9Asset
    from models import GNN, L1Loss
    asset = QM9Asset()
    y = asset.targets[:, :1]
    store = feed.HostStore.from_qm9_asset(asset, precompute_hops=3, threads=2)
    store_t = feed.HostStore.from_arrays(asset.atom_off, asset.bond_off, np.stack([asset.bi, asset.bj], 1),
                                         asset.feats, (y - y.mean()) / y.std(), asset.total_charge, precompute_hops=3)
    del store
    torch.manual_seed(seed)
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, 128, 1, num_shells=3, shell_conv_dropout=dropout, ffn_dropout=dropout).to(DEV).train()
    return store_t, m, L1Loss(), FusedAdam(m.parameters(), lr=1e-3, max_grad_norm=1.0)


def _batches(store, k, B=128, seed=1):
    from aimx import feed
    rng = np.random.default_rng(seed)
    idx = [rng.integers(0, len(store), B) for _ in range(k)]
    c = feed.HostCollator(3, 1)
    sz = np.array([c.plan(store, i) for i in idx])
    f = feed.BatchFeeder(store, iter(idx), 3, DEV, depth=2, n_max=int(sz[:, 0].max()) + 40,
                         e_max=int(sz[:, 1].max()) + 100, pad_mols=8)
    return list(f)


def test_graphed_step_matches_eager_step():
    from aimx.train import GraphedTrainStep, train_step
    store, m1, crit, opt1 = _setup()
    bs = _batches(store, 6)
    _, m2, _, opt2 = _setup()
    m2.load_state_dict(m1.state_dict())
    eager = [train_step(m1, b, crit, opt1, n_real=128)[0].item() for b in bs][1:]
    # one warm-up step on bs[0] (optimizer state, lr upload) mirrors eager's first step
    g = GraphedTrainStep(m2, crit, opt2, bs[0], n_real=128, warmup=1)
    graphed = []
    for b in bs[1:]:
        before = g.loss_sum.item()
        g(b)
        graphed.append((g.loss_sum.item() - before) / 128)
    np.testing.assert_allclose(graphed, eager, rtol=2e-5, atol=1e-6)
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert (p1 - p2).abs().max().item() <= 1e-5 * max(1.0, p1.abs().max().item()), k


def test_training_reduces_loss():
    from aimx.train import GraphedTrainStep, train_epoch
    store, m, crit, opt = _setup(dropout=0.05)
    bs = _batches(store, 12, B=128, seed=3)
    g = GraphedTrainStep(m, crit, opt, bs[0], n_real=128)
    losses = [train_epoch(m, bs, crit, opt, DEV, graphed=g)[0] for _ in range(4)]
    assert losses[-1] < 0.95 * losses[0] and max(losses[1:]) < losses[0], losses
    assert all(np.isfinite(losses))
