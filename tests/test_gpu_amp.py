"""Mixed-precision (AMP) path: the reference's --mixed_precision (trainer.py:134 autocast, 238
GradScaler) on MI355X = bf16 MFMA operands with fp32 accumulation in every node-update / dense GEMM
(AimxGemmArgs.precision = AIMX_PREC_BF16), everything else fp32. fp32 stays the parity path.

Tolerances (stated here):
  * kernel level: against the fp64 product of the bf16-rounded operands, norm-relative 2e-5 (only
    the fp32 accumulation differs), and provably NOT the exact-fp32 product (> 1e-4 away);
  * model level (c2 golden case, forward + backward under torch.autocast): every output and
    parameter gradient within 3e-2 norm-relative of the fp64 oracle — bf16 has an 8-bit mantissa
    (2^-9 relative rounding per operand) — and the loss of a short AMP training run tracks the fp32
    run's."""
import numpy as np
import pytest
import torch

from conftest import norm_rel
from golden_cases import case_stereo, load_case
from test_gpu_parity import _build_model, _gemm, _oracle_run

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K,layout", [
    (9170, 152, 304, "NT"), (9170, 76, 76, "NT"), (1000, 304, 152, "NN"), (2049, 153, 153, "NT"),
    (153, 613, 2000, "TN"), (256, 257, 9186, "TN"), (17, 5, 3, "NT"), (1027, 77, 301, "TT"), (512, 512, 512, "NT")])
def test_gemm_bf16_operands_fp32_accumulate(M, N, K, layout):
    C, _, _, ref, _ = _gemm(M, N, K, layout, bias=True, res=True, prec=1)
    C32, _, _, ref32, _ = _gemm(M, N, K, layout, bias=True, res=True, prec=0)
    if layout == "TN" and K >= 512:
        # a long-K weight gradient (A m-contiguous, B n-contiguous): stays exact fp32 (include/aimx.h)
        assert torch.equal(C, C32)
        return
    err = (C.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-5, err
    if K >= 16:  # the bf16 path really ran: far from the exact fp32 product
        assert (C.double() - ref32).abs().max().item() / ref32.abs().max().item() > 1e-4


def test_model_under_autocast_bf16():
    z, cfg, inputs = load_case("c2")
    torch.set_num_threads(8)
    ref64 = _oracle_run(z, cfg, inputs, torch.float64)
    model = _build_model(cfg, int(z["seed"]))
    af, edges, batch, tc = load_case("c2", DEV)[2]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out, attn, _ = model(af, edges, batch, tc, *case_stereo(z, DEV))
        assert out.dtype == torch.float32
    (out * torch.from_numpy(z["loss_w"]).to(DEV)).sum().backward()
    ours = {"out": out.detach().cpu().numpy(), "attn": attn.detach().cpu().numpy()}
    for k, p in model.named_parameters():
        if p.grad is not None:
            ours["grad." + k] = p.grad.cpu().numpy()
    errs = {k: norm_rel(v, ref64[k]) for k, v in ours.items() if k in ref64}
    for k in [k for k in errs if ".attention_weights." in k and k.endswith(".bias")]:
        # exact value 0 (softmax shift invariance): judged against its weight gradient's scale,
        # as tests/conftest.py parity_failures does
        w = ref64[k[:-len("bias")] + "weight"]
        errs[k] = float(np.abs(ours[k] - ref64[k]).max() / np.abs(w).max())
    assert len(errs) >= 60
    bad = {k: e for k, e in errs.items() if e > 3e-2}
    assert not bad, bad
    assert errs["out"] > 1e-5, "autocast did not switch the GEMMs to bf16 operands"
    # outside autocast the same model is back on the exact fp32 path
    model.zero_grad(set_to_none=True)
    out32, _, _ = model(af, edges, batch, tc, *case_stereo(z, DEV))
    assert norm_rel(out32.detach().cpu().numpy(), ref64["out"]) < 1e-5


def test_amp_training_tracks_fp32():
    """Graph-replayed train steps under autocast (captured inside the autocast context) against the
    fp32 steps (same data, same init, same dropout masks), in two parts:
      * per step, no compounding: at each of the 12 states of the fp32 trajectory, the AMP forward's
        loss (eval mode, no dropout) within 5e-3 relative of the fp32 forward's — bf16 operands
        round at 2^-9 relative and the loss is a mean over 128 molecules;
      * the replayed AMP trajectory itself: its first 6 steps within 1e-2 of fp32's per step, every
        loss finite, and its last 6 steps below its first 6 on average (it trains). Later steps are
        not held per step: Adam's early updates are ~ -lr sign(g), so a gradient entry whose sign
        the bf16 rounding flips moves by 2 lr, and the two trajectories decorrelate (steps 9-11 here
        drift by up to 13 % while step 0-5 agree to 0.5 %).
    The fp32 run itself is pinned tightly (1e-4 per step) to the fp64 oracle's trajectory by
    test_fp32_training_trajectory_matches_oracle."""
    import bench
    from aimx.optim import FusedAdam
    from aimx.train import GraphedTrainStep
    from models import L1Loss
    cfg = dict(bench.CONFIGS["c2"], batch=128)
    bs = bench.make_batches(cfg, 4, 3, DEV, pad=True)
    crit = L1Loss()
    losses, single = {}, []
    for amp in (False, True):
        torch.manual_seed(0)
        m = bench.build_model(cfg, DEV)
        opt = FusedAdam(m.parameters(), lr=1e-3, max_grad_norm=1.0)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            g = GraphedTrainStep(m, crit, opt, bs[0], n_real=128, warmup=1)
        ls = []
        for i in range(12):
            b = bs[i % 4]
            if not amp:  # the AMP forward's error at this fp32 state alone
                m.eval()
                with torch.no_grad():
                    l32 = crit(m(*b.model_args())[0][:128], b.targets[:128]).item()
                    with torch.autocast("cuda", dtype=torch.bfloat16):
                        l16 = crit(m(*b.model_args())[0][:128], b.targets[:128]).item()
                m.train()
                single.append(abs(l16 - l32) / l32)
            before = g.loss_sum.item()
            g(b)
            ls.append((g.loss_sum.item() - before) / 128)
        losses[amp] = np.array(ls)
    assert max(single) <= 5e-3, single
    assert min(single) > 0, "autocast did not switch the GEMMs to bf16 operands"
    assert np.all(np.isfinite(losses[True]))
    np.testing.assert_allclose(losses[True][:6], losses[False][:6], rtol=1e-2, atol=0)
    for amp in (False, True):
        assert losses[amp][6:].mean() < losses[amp][:6].mean(), (amp, losses[amp])


def test_fp32_training_trajectory_matches_oracle():
    """The fp32 pin the AMP comparison above leans on: 12 graph-replayed train steps (forward, L1,
    backward, clip(1.0), Adam lr 1e-3; dropout off) on 4 resampled QM9 batches of 128 molecules
    against the same 12 steps of the oracle in fp64 with torch's own clip_grad_norm_ and Adam, from
    the same initial weights: every step's loss within 1e-4 relative. (The bf16 run above is held
    only to 2 % in the mean / 10 % per step: bf16 operand rounding, 2^-9 relative, compounds
    through Adam's updates — that looser bound applies to AMP alone.)"""
    import bench
    from aimx.optim import FusedAdam
    from aimx.train import GraphedTrainStep
    from models import GNN, L1Loss
    from oracle import model as om
    cfg = dict(bench.CONFIGS["c2"], batch=128)
    bs = bench.make_batches(cfg, 4, 3, DEV, pad=True)
    cols = bench.make_collated(cfg, 4, 3)  # the same molecules, unpadded (same seed)
    torch.manual_seed(0)
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, 256, 1, num_shells=3, shell_conv_dropout=0.0, ffn_dropout=0.0).to(DEV).train()
    m.init_weights()
    init = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}
    opt = FusedAdam(m.parameters(), lr=1e-3, max_grad_norm=1.0)
    g = GraphedTrainStep(m, L1Loss(), opt, bs[0], n_real=128, warmup=1)
    ours = []
    for i in range(12):
        before = g.loss_sum.item()
        g(bs[i % 4])
        ours.append((g.loss_sum.item() - before) / 128)
    ocfg = om.default_config(hidden_dim=256, num_shells=3, output_dim=1)
    p = {k: v.clone().requires_grad_() for k, v in init.items()}
    aopt = torch.optim.Adam(p.values(), lr=1e-3)
    torch.set_num_threads(8)
    ref = []
    for i in range(12):
        col, tg, q = cols[i % 4]
        feats = torch.from_numpy(col["feats"].astype(np.int64))
        af = {k: feats[:, j].contiguous() for j, k in enumerate(("atom_type", "hydrogen_count", "degree",
                                                                  "hybridization"))}
        aopt.zero_grad(set_to_none=True)
        out, _, _ = om.gnn_forward(p, ocfg, af, torch.from_numpy(col["edges"].astype(np.int64)).reshape(-1, 2),
                                   torch.from_numpy(col["batch"].astype(np.int64)), torch.from_numpy(q).double())
        loss = torch.nn.functional.l1_loss(out, torch.from_numpy(tg).double())
        loss.backward()
        torch.nn.utils.clip_grad_norm_([v for v in p.values() if v.grad is not None], 1.0)
        aopt.step()
        ref.append(loss.item())
    np.testing.assert_allclose(ours, ref, rtol=1e-4, atol=0)
