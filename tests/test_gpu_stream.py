"""GPU: the c5-shaped stream leg end to end. A 6-hop file of synthetic 40-atom molecules in the
reference's HDF5 dataset format (features.py:381-431) is read by HDF5MolecularStream (the native
counterpart of HDF5MolecularIterableDataset, molecular.py:102-329: shuffled positions, equal rank
shards), collated by the C++ batch builder and copied host->device by BatchFeeder, then run through
the GPU GNN (c5s architecture: hidden 1024, 6 hops, attention pool) forward and backward. Checked
against an independent path: the same molecules regenerated from their seeds, collated by the
Python restatement (bit-exact edges / batch / features) and run through the fp64 / fp32 oracle."""
import numpy as np
import pytest
import torch

from conftest import parity_failures
from golden_cases import FEATURE_KEYS, load_case, reversed_molecules
from test_gpu_parity import _build_model

pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED = 7


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import aimx
    aimx.load()


def _oracle_grads(cfg, seed, af, edges, batch, tc, loss_w, dtype):
    from oracle import model as om
    p = {k: v.to(dtype).requires_grad_() for k, v in om.seeded_params(cfg, seed).items()}
    cap = {}
    out, attn, _ = om.gnn_forward(p, cfg, af, edges, batch, tc.to(dtype), capture=cap)
    (out * torch.from_numpy(loss_w).to(dtype)).sum().backward()
    res = {"grad." + k: v.grad.numpy() for k, v in p.items() if v.grad is not None}
    res.update(out=out.detach().numpy(), attn=attn.detach().numpy())
    if dtype == torch.float64:  # the temperature gradient's term scale (conftest._scale_for)
        res["scale:grad.pooling.temperature"] = om.temperature_scale(cap)
    return res


@pytest.mark.parametrize("world,rank", [(1, 0), (2, 1)])
def test_stream_6hop_feeds_gpu_model_at_parity(tmp_path, world, rank):
    from aimx import data as adata
    from aimx import feed, h5
    from aimx.synth import synth_molecule
    z, cfg, _ = load_case("c5s")
    hops, B, n_mols = cfg["num_shells"], 24, 80
    assert hops == 6
    path = str(tmp_path / "stream6.h5")
    h5.make_synthetic_stream(path, n_mols, "synth40", hops=hops, tasks=1, seed=SEED, workers=2, chunk=32)
    stream = h5.HDF5MolecularStream(path, shuffle=True, ddp_enabled=world > 1, rank=rank, world_size=world,
                                    n_hops=hops, n_tasks=1, threads=2)
    pos = stream.positions(epoch_seed=3)
    assert len(pos) == (n_mols + world - 1) // world
    fed = feed.BatchFeeder(None, stream.batches(B, chunk_size=n_mols, epoch_seed=3), hops, DEV, depth=2, threads=2)
    model = _build_model(cfg, int(z["seed"]))
    torch.set_num_threads(8)
    seen = 0
    for j, b in enumerate(fed):
        recs = pos[j * B:(j + 1) * B]
        mols = [synth_molecule(np.random.default_rng([SEED, int(k)])) for k in recs]
        col = adata.collate(mols, hops)
        # the native reader + batch builder deliver exactly the Python-collated batch
        assert torch.equal(b.edges.cpu(), torch.from_numpy(col["edges"].astype(np.int64)).reshape(-1, 2))
        assert torch.equal(b.batch.cpu(), torch.from_numpy(col["batch"].astype(np.int64)))
        feats = torch.from_numpy(col["feats"].astype(np.int64))
        for i, k in enumerate(FEATURE_KEYS):
            assert torch.equal(b.atom_features[k].cpu(), feats[:, i]), k
        assert b.real_graphs == len(recs) == B
        loss_w = np.random.default_rng(j).standard_normal((B, cfg["output_dim"])).astype(np.float32)
        for p in model.parameters():
            p.grad = None
        out, attn, _ = model(*b.model_args())
        (out * torch.from_numpy(loss_w).to(DEV)).sum().backward()
        ours = {"out": out.detach().cpu().numpy(), "attn": attn.detach().cpu().numpy()}
        ours.update({"grad." + k: p.grad.cpu().numpy() for k, p in model.named_parameters() if p.grad is not None})
        af = {k: feats[:, i].contiguous() for i, k in enumerate(FEATURE_KEYS)}
        edges = torch.from_numpy(col["edges"].astype(np.int64)).reshape(-1, 2)
        batch = torch.from_numpy(col["batch"].astype(np.int64))
        tc = torch.zeros(B)
        ref64 = _oracle_grads(cfg, int(z["seed"]), af, edges, batch, tc, loss_w, torch.float64)
        ref32 = _oracle_grads(cfg, int(z["seed"]), af, edges, batch, tc, loss_w, torch.float32)
        (raf, red, rb, rtc), rlw, unperm = reversed_molecules((af, edges, batch, tc), loss_w)
        ref32r = unperm(_oracle_grads(cfg, int(z["seed"]), raf, red, rb, rtc, rlw, torch.float32))
        assert set(ours) == {k for k in ref64 if not k.startswith("scale:")}
        bad = parity_failures(ours, None, ref64, oracle32=[ref32, ref32r])
        assert not bad, bad
        seen += 1
    assert seen == len(pos) // B >= 1
