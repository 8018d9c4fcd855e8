"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and the oracle.

Integer work (CSR / edge order) bit-exact; the hop forward bit-exact (same summation order as the
reference's CPU scatter_add_); floating point per tensor within the north-star tolerance
(conftest.parity_failures: <= max(1e-5, 3x the reference's own fp32 error vs fp64)).
"""
import os

import numpy as np
import pytest
import torch

from conftest import add_sketches, fixture_refs, load_golden, norm_rel, parity_failures
from golden_cases import CASES, case_stereo, load_case, reversed_molecules

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import aimx
    aimx.load()


def _oracle():
    from oracle import graph as og
    from oracle import model as om
    return og, om


# ------------------------------------------------------------------------------------------ CSR
@pytest.mark.parametrize("case", ["c1", "c2", "c3", "c5s"])
def test_csr_bit_exact(case):
    from aimx.plan import GraphPlan
    og, _ = _oracle()
    z = load_golden(case)
    edges = torch.from_numpy(z["edges"].astype(np.int64)).to(DEV)
    batch = torch.from_numpy(z["batch"].astype(np.int64)).to(DEV)
    n = z["feats"].shape[0]
    h = 6 if case == "c5s" else (4 if case == "c3" else 3)
    g = len(z["n_mol_atoms"])
    plan = GraphPlan(n, h, edges=edges, batch=batch, num_graphs=g)
    e = z["edges"].astype(np.int64)
    rp, col = og.stable_csr(e[:, 0], np.mod(e[:, 1], n), h * n)
    assert np.array_equal(plan.fwd.rowptr.cpu().numpy(), rp)
    assert np.array_equal(plan.fwd.col.cpu().numpy()[: len(col)], col)
    rp, col = og.stable_csr(np.mod(e[:, 1], n), e[:, 0], n)
    assert np.array_equal(plan.bwd.rowptr.cpu().numpy(), rp)
    assert np.array_equal(plan.bwd.col.cpu().numpy()[: len(col)], col)
    rp, col = og.stable_csr(z["batch"].astype(np.int64), np.arange(n), g)
    assert np.array_equal(plan.graph.rowptr.cpu().numpy(), rp)
    assert np.array_equal(plan.graph.col.cpu().numpy()[: len(col)], col)
    assert int(plan.status.item()) == 0


def test_csr_general_and_out_of_range():
    from aimx.plan import GraphPlan
    og, _ = _oracle()
    rng = np.random.default_rng(3)
    n, h, e = 1000, 4, 50000
    t = rng.integers(0, h * n, e)
    s = rng.integers(-5 * n, 5 * n, e)
    plan = GraphPlan(n, h, target=torch.from_numpy(t).to(DEV), src=torch.from_numpy(s).to(DEV))
    rp, col = og.stable_csr(t, np.mod(s, n), h * n)
    assert np.array_equal(plan.fwd.rowptr.cpu().numpy(), rp)
    assert np.array_equal(plan.fwd.col.cpu().numpy(), col)
    assert int(plan.status.item()) == 0
    t2 = t.copy()
    t2[7] = h * n + 3  # the reference would raise: flagged and dropped, never a fault
    plan = GraphPlan(n, h, target=torch.from_numpy(t2).to(DEV), src=torch.from_numpy(s).to(DEV))
    assert int(plan.status.item()) == 1
    with pytest.raises(RuntimeError):
        plan.validate()


def test_csr_large_rows_multiblock_scan():
    from aimx.plan import GraphPlan
    og, _ = _oracle()
    rng = np.random.default_rng(4)
    n, h, e = 700_000, 3, 2_000_000
    t = rng.integers(0, h * n, e)
    s = rng.integers(0, n, e)
    plan = GraphPlan(n, h, target=torch.from_numpy(t).to(DEV), src=torch.from_numpy(s).to(DEV))
    rp, col = og.stable_csr(t, s, h * n)
    assert np.array_equal(plan.fwd.rowptr.cpu().numpy(), rp)
    assert np.array_equal(plan.fwd.col.cpu().numpy(), col)


# ------------------------------------------------------------------------------------------ hop
def test_hop_forward_bit_exact_general():
    """Hop-offset targets, src >= N and negative src (the general layers.py:133-167 contract)."""
    from models.layers import ShellConvolutionLayer
    z = load_golden("mp_general")
    layer = ShellConvolutionLayer(38, 38, num_hops=3).to(DEV)
    x = torch.from_numpy(z["x"]).to(DEV)
    chunks = layer.message_passing(x, torch.from_numpy(z["tgt"]).to(DEV), torch.from_numpy(z["src"]).to(DEV))
    assert np.array_equal(torch.cat(chunks, 0).cpu().numpy(), z["chunks"])


@pytest.mark.parametrize("d", [38, 76, 153, 307, 64, 2])
def test_hop_forward_bit_exact_widths(d):
    """Every vector width path (float4 / float2 / scalar) is bit-exact vs CPU scatter_add_."""
    from aimx.plan import GraphPlan
    from aimx import ops
    _, om = _oracle()
    z = load_golden("c2")
    e = torch.from_numpy(z["edges"].astype(np.int64))
    n = z["feats"].shape[0]
    x = torch.randn(n, d, generator=torch.Generator().manual_seed(d))
    ref = torch.cat(om.message_passing(x, e[:, 0], e[:, 1], 3), 0)
    plan = GraphPlan(n, 3, edges=e.to(DEV))
    out = ops.hop(plan, x.to(DEV))
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("hub_degree", [9, 300, 20_000])
def test_hop_forward_bit_exact_hubs(hub_degree):
    """Ragged degrees: rows longer than one 8-gather group and row tiles whose edge list exceeds the
    LDS staging capacity (global col path); empty rows and empty tiles in between; backward too."""
    from aimx.plan import GraphPlan
    from aimx import ops
    _, om = _oracle()
    rng = np.random.default_rng(hub_degree)
    n, h = 3000, 3
    base_t = rng.integers(0, n, 20_000)
    hubs = rng.choice(n, 5, replace=False)
    t = np.concatenate([base_t, np.repeat(hubs, hub_degree)])
    s = rng.integers(-n, 2 * n, t.shape[0])
    perm = rng.permutation(t.shape[0])
    t, s = torch.from_numpy(t[perm]), torch.from_numpy(s[perm])
    x = torch.randn(n, 76, generator=torch.Generator().manual_seed(3))
    ref = torch.cat(om.message_passing(x, t, s, h), 0)
    plan = GraphPlan(n, h, target=t.to(DEV), src=s.to(DEV))
    xg = x.to(DEV).requires_grad_()
    out = ops.hop(plan, xg)
    assert torch.equal(out.detach().cpu(), ref)
    w = torch.randn(ref.shape, generator=torch.Generator().manual_seed(4))
    (out * w.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_()
    (torch.cat(om.message_passing(x64, t, s, h), 0) * w.double()).sum().backward()
    assert norm_rel(xg.grad.cpu().numpy(), x64.grad.numpy()) < 1e-6


def test_hop_forward_bit_exact_large():
    """A multi-molecule graph with rows * D >= 2^24 (thousands of row tiles): still bit-exact."""
    from aimx.plan import GraphPlan
    from aimx import ops
    _, om = _oracle()
    z = load_golden("c2")
    e0 = torch.from_numpy(z["edges"].astype(np.int64))
    n0 = z["feats"].shape[0]
    reps = 9
    e = torch.cat([e0 + r * n0 for r in range(reps)], 0)
    n = n0 * reps
    assert 3 * n * 76 >= 1 << 24
    x = torch.randn(n, 76, generator=torch.Generator().manual_seed(5))
    ref = torch.cat(om.message_passing(x, e[:, 0], e[:, 1], 3), 0)
    plan = GraphPlan(n, 3, edges=e.to(DEV))
    out = ops.hop(plan, x.to(DEV))
    assert torch.equal(out.cpu(), ref)


def test_hop_backward():
    from aimx.plan import GraphPlan
    from aimx import ops
    _, om = _oracle()
    z = load_golden("mp_general")
    x = torch.from_numpy(z["x"]).double().requires_grad_()
    t, s = torch.from_numpy(z["tgt"]), torch.from_numpy(z["src"])
    ref = torch.cat(om.message_passing(x, t, s, 3), 0)
    w = torch.randn(ref.shape, dtype=torch.float64, generator=torch.Generator().manual_seed(1))
    (ref * w).sum().backward()
    xg = torch.from_numpy(z["x"]).to(DEV).requires_grad_()
    plan = GraphPlan(50, 3, target=t.to(DEV), src=s.to(DEV))
    out = ops.hop(plan, xg)
    (out * w.float().to(DEV)).sum().backward()
    assert norm_rel(xg.grad.cpu().numpy(), x.grad.numpy()) < 1e-6


# ----------------------------------------------------------------------------------------- GEMM
def _gemm(M, N, K, layout, **epi):
    """Run aimx_gemm on random data; returns (C_gpu, inputs) for checking against torch fp64."""
    import ctypes
    from aimx import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g) if layout[0] == "N" else torch.randn(K, M, generator=g)
    B = torch.randn(K, N, generator=g) if layout[1] == "N" else torch.randn(N, K, generator=g)
    if "A" in epi:
        A = epi["A"]
    if "B" in epi:
        B = epi["B"]
    Ad, Bd = A.to(DEV), B.to(DEV)
    ones = epi.get("ones", False)
    Nt = N + 1 if ones else N
    C = torch.zeros(M, N, device=DEV)
    col = torch.zeros(M, device=DEV)
    a = _lib.GemmArgs()
    a.M, a.N, a.K = M, Nt, K
    a.A = Ad.data_ptr()
    a.sam, a.sak = (K, 1) if layout[0] == "N" else (1, M)
    a.B = Bd.data_ptr()
    a.sbk, a.sbn = (N, 1) if layout[1] == "N" else (1, K)
    a.C, a.ldc = C.data_ptr(), N
    a.act, a.dact_kind = -1, -1
    bias = torch.randn(N, generator=g).to(DEV) if epi.get("bias") else None
    if bias is not None:
        a.bias = bias.data_ptr()
    pre = torch.zeros(M, N, device=DEV)
    if epi.get("act") is not None:
        a.act, a.act_ncols, a.pre, a.ldpre = epi["act"], N, pre.data_ptr(), N
    res = torch.randn(M, N, generator=g).to(DEV) if epi.get("res") else None
    if res is not None:
        a.res[0], a.ldres[0] = res.data_ptr(), N
    if ones:
        a.ones_col, a.col_out = 1, col.data_ptr()
    dpre = torch.randn(M, N, generator=g).to(DEV) if epi.get("dact") is not None else None
    if dpre is not None:  # input-gradient epilogue: C = (AB) * act'(dpre) [* mask / (1 - p)]
        a.dact_pre, a.lddact, a.dact_kind = dpre.data_ptr(), N, epi["dact"]
    mask = (torch.rand(M, N, generator=g) > 0.3).to(torch.uint8).to(DEV) if epi.get("mask") else None
    if mask is not None:
        a.mask_in, a.ldmask, a.drop_p = mask.data_ptr(), N, 0.3
    a.splits = epi.get("splits", 0)
    a.precision = epi.get("prec", 0)
    if epi.get("zc") is not None:
        rp, rows, chunks, width, dim = epi["zc"]
        a.zc_rowptr, a.zc_rows, a.zc_chunks, a.zc_width, a.zc_dim = rp.data_ptr(), rows, chunks, width, dim
    if epi.get("fused_reduce", True):
        a.counters, a.n_counters = _lib.counters(DEV).data_ptr(), _lib.N_COUNTERS
    wsb = lib.aimx_gemm_workspace_bytes(ctypes.byref(a))
    ws = torch.empty(max(wsb // 4, 1) + 64 * 1024, device=DEV)
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    assert lib.aimx_gemm(ctypes.byref(a), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    Am = A if layout[0] == "N" else A.t()
    Bm = B if layout[1] == "N" else B.t()
    if epi.get("prec", 0) == 1:  # bf16 operands (RNE), exact products accumulated in fp64 here
        ref = Am.to(torch.bfloat16).double() @ Bm.to(torch.bfloat16).double()
    else:
        ref = Am.double() @ Bm.double()
    if bias is not None:
        ref = ref + bias.cpu().double()
    if res is not None:
        ref = ref + res.cpu().double()
    if dpre is not None:
        x = dpre.cpu().double()
        sg = torch.sigmoid(x)
        assert epi["dact"] == 4  # silu'
        ref = ref * (sg * (1 + x * (1 - sg)))
    if mask is not None:
        ref = ref * mask.cpu().double() / 0.7
    return C.cpu(), col.cpu(), pre.cpu(), ref, Am


@pytest.mark.parametrize("M,N,K,layout", [
    (9170, 152, 304, "NT"), (9170, 76, 76, "NT"), (1000, 304, 152, "NN"), (153, 613, 2000, "TN"),
    (17, 5, 3, "NT"), (64, 64, 16, "NN"), (307, 307, 10240, "TN"), (100, 2149, 614, "NN"),
    (1, 513, 512, "TN"), (512, 1, 512, "NT"), (3, 7, 1, "NN"),
    (76, 78, 9170, "TN"), (33, 65, 701, "TN"), (5, 3, 515, "TN"), (256, 257, 9186, "TN")])
def test_gemm_layouts(M, N, K, layout):
    C, _, _, ref, _ = _gemm(M, N, K, layout, bias=True, res=True)
    err = (C.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


@pytest.mark.parametrize("M,N,K,layout,splits", [
    (258, 1024, 1024, "NT", 0), (258, 1024, 1024, "NN", 0), (256, 512, 1000, "NT", 0), (1, 256, 256, "NN", 0),
    (640, 260, 300, "NT", 0), (130, 1024, 4096, "NN", 0), (64, 256, 256, "NT", 0), (200, 516, 260, "NN", 0),
    (258, 1024, 1024, "NT", 1), (258, 1024, 1024, "NN", 7), (77, 300, 1028, "NT", 64)])
def test_gemm_few_rows_deep_k(M, N, K, layout, splits):
    """Few rows, wide and deep (c5's post-pool F = 1024 layers and their input gradient: 32 x 32
    tiles split over K): padded row blocks, N and K tails, one split and forced split counts;
    against fp64, deterministic (bitwise) and counters left at zero."""
    from aimx import _lib
    C, _, _, ref, _ = _gemm(M, N, K, layout, bias=True, res=True, splits=splits)
    err = (C.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    C2, _, _, _, _ = _gemm(M, N, K, layout, bias=True, res=True, splits=splits)
    assert torch.equal(C, C2)
    assert int(_lib.counters(DEV).abs().sum().item()) == 0


@pytest.mark.parametrize("M,N,K,ones", [(1024, 1024, 258, True), (1024, 1024, 258, False), (512, 512, 516, True),
                                        (260, 300, 1000, True), (1024, 256, 61, True), (256, 1020, 7, False)])
def test_gemm_short_k_weight_gradient(M, N, K, ones):
    """Short-K weight gradients (dW = dY^T X: A m-contiguous, B n-contiguous; the post-pool chain's
    F x F at K = molecules) with the implicit ones column (bias gradient): K tails, a partial last
    column block holding only the ones column; fp64, bitwise deterministic."""
    C, col, _, ref, Am = _gemm(M, N, K, "TN", ones=ones)
    assert (C.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    if ones:
        rs = Am.double().sum(1)
        assert (col.double() - rs).abs().max().item() / rs.abs().max().item() < 2e-6
    C2, col2, _, _, _ = _gemm(M, N, K, "TN", ones=ones)
    assert torch.equal(C, C2) and torch.equal(col, col2)


@pytest.mark.parametrize("M,N,K,layout", [(256, 1024, 1024, "NT"), (256, 1024, 1024, "NN"), (257, 1000, 1028, "NT"),
                                          (256, 12, 2048, "NT"), (1, 4100, 512, "NN"), (1024, 64, 516, "NN"),
                                          (96, 1024, 4100, "NT")])
@pytest.mark.parametrize("deep", [16, 8, 0])
def test_gemm_deep_kernel(M, N, K, layout, deep):
    """k_gemm_deep (8 waves per 32 x 32 tile, each 1/8 of K from a register ring, summed in wave
    order) against fp64 and against the LDS-staged tiles (AIMX_GEMM_DEEP option 0): the c5 head's
    forward ([n][k] weights) and input gradient ([k][n]), row / column / K % 8 == 4 tails, the
    output layer (N = T: the tiles' rule, too few tiles for the deep kernel), one row; the epilogues (bias + residual, SiLU with the pre-activation
    store, the input gradient's act'(pre) x dropout mask); bitwise deterministic."""
    from aimx import _lib
    with _lib.options(AIMX_GEMM_DEEP=deep):
        C, _, _, ref, _ = _gemm(M, N, K, layout, bias=True, res=True)
        C2, _, _, _, _ = _gemm(M, N, K, layout, bias=True, res=True)
        Ca, _, pre, refa, _ = _gemm(M, N, K, layout, bias=True, act=4)
        Cg, _, _, refg, _ = _gemm(M, N, K, layout, dact=4, mask=True)
    assert (C.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    assert torch.equal(C, C2)
    assert (pre.double() - refa).abs().max().item() / refa.abs().max().item() < 2e-6
    fr = torch.nn.functional.silu(refa)
    assert (Ca.double() - fr).abs().max().item() / fr.abs().max().item() < 2e-6
    assert (Cg.double() - refg).abs().max().item() / refg.abs().max().item() < 2e-6


def test_gemm_deep_k_activation_epilogue():
    C, _, pre, ref, _ = _gemm(258, 1024, 1024, "NT", bias=True, act=4)
    assert (pre.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    fr = torch.nn.functional.silu(ref)
    assert (C.double() - fr).abs().max().item() / fr.abs().max().item() < 2e-6


def _gemm_raw(M, N, K, layout, off, pa, pb, ones=False):
    """aimx_gemm on operands that start `off` floats into their buffers with row strides padded by
    pa / pb floats; returns (C, bias-gradient column, fp64 reference)."""
    import ctypes
    from aimx import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K + off)
    rA, cA = (M, K) if layout[0] == "N" else (K, M)
    rB, cB = (K, N) if layout[1] == "N" else (N, K)
    la, lb = cA + pa, cB + pb
    bufA = torch.randn(off + rA * la, generator=g)
    bufB = torch.randn(off + rB * lb, generator=g)
    A = bufA[off:].view(rA, la)[:, :cA]
    B = bufB[off:].view(rB, lb)[:, :cB]
    dA, dB = bufA.to(DEV), bufB.to(DEV)
    C = torch.zeros(M, N, device=DEV)
    col = torch.zeros(M, device=DEV)
    a = _lib.GemmArgs()
    a.M, a.N, a.K = M, N + (1 if ones else 0), K
    a.A = dA.data_ptr() + 4 * off
    a.sam, a.sak = (la, 1) if layout[0] == "N" else (1, la)
    a.B = dB.data_ptr() + 4 * off
    a.sbk, a.sbn = (lb, 1) if layout[1] == "N" else (1, lb)
    a.C, a.ldc = C.data_ptr(), N
    a.act, a.dact_kind = -1, -1
    if ones:
        a.ones_col, a.col_out = 1, col.data_ptr()
    a.counters, a.n_counters = _lib.counters(DEV).data_ptr(), _lib.N_COUNTERS
    wsb = lib.aimx_gemm_workspace_bytes(ctypes.byref(a))
    ws = torch.empty(max(wsb // 4, 1) + 64 * 1024, device=DEV)
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    assert lib.aimx_gemm(ctypes.byref(a), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    Am = A if layout[0] == "N" else A.t()
    Bm = B if layout[1] == "N" else B.t()
    return C.cpu(), col.cpu(), Am.double() @ Bm.double(), Am


@pytest.mark.parametrize("M,N,K,layout,off,pa,pb,ones", [
    (2049, 153, 153, "NT", 1, 0, 0, False), (2049, 153, 153, "NN", 2, 3, 0, False), (1003, 307, 307, "NT", 3, 0, 1, False),
    (1003, 307, 306, "NN", 0, 1, 2, False), (517, 77, 153, "NT", 1, 0, 0, True), (33, 5, 3, "NT", 2, 0, 0, False),
    (700, 153, 31, "NT", 3, 2, 0, False), (64, 160, 614, "NT", 1, 1, 3, False), (300, 45, 153, "TT", 2, 1, 0, False)])
def test_gemm_unaligned_rows_ones_column(M, N, K, layout, off, pa, pb, ones):
    """The dword staging of unaligned k-contiguous operands (c4/c5's D = 153 / 307 rows): odd widths
    and row strides, every base misalignment, K tails shorter than a slice, the ones column; within
    2e-6 of fp64 and bitwise deterministic."""
    C1, col1, ref, Am = _gemm_raw(M, N, K, layout, off, pa, pb, ones)
    C0, col0, _, _ = _gemm_raw(M, N, K, layout, off, pa, pb, ones)
    assert torch.equal(C1, C0) and torch.equal(col1, col0)
    err = (C1.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    if ones:
        rs = Am.double().sum(1)
        assert (col1.double() - rs).abs().max().item() / rs.abs().max().item() < 2e-6


@pytest.mark.parametrize("M,N,K,layout,off", [(2049, 153, 153, "NT", 1), (2049, 307, 153, "NN", 3),
                                               (153, 307, 4099, "TN", 2), (1027, 77, 301, "TT", 1),
                                               (5, 3, 7, "NT", 3)])
def test_gemm_unaligned_rows_and_bases(M, N, K, layout, off):
    """16-byte staging at any float alignment: operands are views starting `off` floats into their
    buffers with odd row strides (the c4/c5 widths D = 153 / 307), so rows, bases and the extent's
    last float4 are all misaligned."""
    import ctypes
    from aimx import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K)
    rA, cA = (M, K) if layout[0] == "N" else (K, M)
    rB, cB = (K, N) if layout[1] == "N" else (N, K)
    la, lb = cA + 3, cB + 1
    bufA = torch.randn(off + rA * la, generator=g)
    bufB = torch.randn(off + rB * lb, generator=g)
    A = bufA[off:].view(rA, la)[:, :cA]
    B = bufB[off:].view(rB, lb)[:, :cB]
    dA, dB = bufA.to(DEV), bufB.to(DEV)
    C = torch.zeros(M, N, device=DEV)
    a = _lib.GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.A = dA.data_ptr() + 4 * off
    a.sam, a.sak = (la, 1) if layout[0] == "N" else (1, la)
    a.B = dB.data_ptr() + 4 * off
    a.sbk, a.sbn = (lb, 1) if layout[1] == "N" else (1, lb)
    a.C, a.ldc = C.data_ptr(), N
    a.act, a.dact_kind = -1, -1
    a.counters, a.n_counters = _lib.counters(DEV).data_ptr(), _lib.N_COUNTERS
    wsb = lib.aimx_gemm_workspace_bytes(ctypes.byref(a))
    ws = torch.empty(max(wsb // 4, 1) + 64 * 1024, device=DEV)
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    assert lib.aimx_gemm(ctypes.byref(a), torch.cuda.current_stream().cuda_stream) == 0
    Am = A if layout[0] == "N" else A.t()
    Bm = B if layout[1] == "N" else B.t()
    ref = Am.double() @ Bm.double()
    err = (C.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


@pytest.mark.parametrize("M,N,K,layout,off,pa,pb", [
    (10240, 614, 614, "NT", 0, 1538, 1535),   # c5 [u|g]: F rows of ld 2152, weight rows of 2149 (odd)
    (10241, 2149, 614, "NN", 1, 2, 0),         # c5 input gradient: B n-contiguous, N tail, odd base
    (10240, 1024, 1024, "NT", 0, 0, 0),        # c5 concat
    (20481, 306, 306, "NT", 3, 306, 306),      # c4 [u|g] (K tail inside a float4 and a slice)
    (9999, 512, 257, "NN", 2, 1, 3),           # K % 32 = 1, every base misaligned
    (4096, 130, 3000, "NT", 1, 0, 1)])         # deep K, a 2-column tail tile
def test_gemm_config_shapes_unaligned(M, N, K, layout, off, pa, pb):
    """The c4 / c5 projections and input gradients at their row strides: odd row strides and bases (16-byte loads at 4-byte alignment), M / N / K tails, both B
    layouts; within 3e-6 of fp64 (the max error relative to the max entry: K = 3000 accumulates
    2.3e-6) and bitwise deterministic."""
    C, _, ref, _ = _gemm_raw(M, N, K, layout, off, pa, pb)
    C2, _, _, _ = _gemm_raw(M, N, K, layout, off, pa, pb)
    assert torch.isfinite(C).all()
    err = (C.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 3e-6, err
    assert torch.equal(C, C2)


@pytest.mark.parametrize("M,N,K,ones", [(1024, 1024, 10240, True), (512, 512, 20480, True), (307, 307, 4099, True),
                                        (130, 70, 2049, False), (256, 257, 9170, True)])
def test_gemm_long_k_weight_gradient(M, N, K, ones):
    """Long-K weight gradients (dW = dY^T X: A m-contiguous, B n-contiguous, K = atoms split over
    workgroups with an ordered slab reduction by the last arriver) with the implicit ones column
    (the bias gradient): the c4 / c5 concat and embedding shapes, c5's 307-wide MLP weights, small
    odd shapes; within 2e-6 of fp64, bitwise deterministic, counters left at zero."""
    from aimx import _lib
    C, col, _, ref, Am = _gemm(M, N, K, "TN", ones=ones)
    C2, col2, _, _, _ = _gemm(M, N, K, "TN", ones=ones)
    assert torch.isfinite(C).all()
    assert (C.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    if ones:
        rs = Am.double().sum(1)
        assert (col.double() - rs).abs().max().item() / rs.abs().max().item() < 2e-6
    assert torch.equal(C, C2) and torch.equal(col, col2)
    assert int(_lib.counters(DEV).abs().sum().item()) == 0


def test_gemm_weight_gradient_trimming_c5():
    """The weight gradient over F with empty hop chunks (zc_dim 1) at c5's width: blocks wholly past
    E are written as zeros without loads, the block straddling E reads F's columns past E as 0 (they
    hold NaN here: the stack's hop leaves them unwritten); equal to the untrimmed product bitwise."""
    n, d, h = 12000, 307, 6
    K = d * (h + 1)
    counts = torch.zeros(h * n, dtype=torch.int32)
    counts[0:n:5] = 3
    rowptr = torch.cat([torch.zeros(1, dtype=torch.int32), counts.cumsum(0).to(torch.int32)]).to(DEV)
    E = 2 * d
    g = torch.Generator().manual_seed(13)
    F = torch.randn(n, K, generator=g)
    F[:, E:] = 0
    Fnan = F.clone()
    Fnan[:, E:] = float("nan")
    dY = torch.randn(n, 2 * d, generator=g)
    full, fcol, _, ref, _ = _gemm(2 * d, K, n, "TN", A=dY, B=F, ones=True)
    trim, tcol, _, _, _ = _gemm(2 * d, K, n, "TN", A=dY, B=Fnan, ones=True, zc=(rowptr, n, h, d, 1))
    assert torch.equal(full, trim) and torch.equal(fcol, tcol)
    assert not trim[:, E:].any()
    assert (full.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6


def test_gemm_epilogue_and_trimming_c5():
    """The fused epilogue (bias, residual, SiLU with the pre-activation store) and the
    empty-hop-chunk trimming at c5 size: forward k loop stopped at E (NaN past it is never read) equals
    the untrimmed product bitwise; the input gradient's tiles past E are skipped (zc_dim 2) and every
    column < E is bitwise the untrimmed one."""
    n, d, h = 10240, 307, 6
    K = d * (h + 1)
    C, _, pre, ref, _ = _gemm(n, 2 * d, 1024, "NT", bias=True, act=4, res=True)
    assert (pre.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    fr = torch.nn.functional.silu(ref)  # bias and residual enter the pre-activation (epi_apply)
    assert (C.double() - fr).abs().max().item() / fr.abs().max().item() < 2e-6
    counts = torch.zeros(h * n, dtype=torch.int32)
    counts[0:n:5] = 3
    rowptr = torch.cat([torch.zeros(1, dtype=torch.int32), counts.cumsum(0).to(torch.int32)]).to(DEV)
    E = 2 * d
    g = torch.Generator().manual_seed(9)
    F = torch.randn(n, K, generator=g)
    F[:, E:] = 0
    Fnan = F.clone()
    Fnan[:, E:] = float("nan")
    W = torch.randn(2 * d, K, generator=g)
    full, _, _, ref2, _ = _gemm(n, 2 * d, K, "NT", A=F, B=W)
    trim, _, _, _, _ = _gemm(n, 2 * d, K, "NT", A=Fnan, B=W, zc=(rowptr, n, h, d, 0))
    assert torch.equal(full, trim)
    assert (trim.double() - ref2).abs().max().item() / ref2.abs().max().item() < 2e-6
    dUG = torch.randn(n, 2 * d, generator=g)
    full, _, _, _, _ = _gemm(n, K, 2 * d, "NN", A=dUG, B=W)
    trim, _, _, _, _ = _gemm(n, K, 2 * d, "NN", A=dUG, B=W, zc=(rowptr, n, h, d, 2))
    assert torch.equal(full[:, :E], trim[:, :E])


@pytest.mark.parametrize("d", [76, 153])
@pytest.mark.parametrize("nonempty", [(True, False, False), (False, False, False), (True, True, False),
                                      (False, True, False), (True, False, True)])
def test_gemm_empty_hop_chunk_trimming(nonempty, d):
    """zc_* trimming (the reference's all-zero hop chunks, layers.py:154): F = [x | c0 | c1 | c2]
    with the empty chunks zero. Forward (k loop stops at E) and weight gradient (zero tiles) equal
    the untrimmed products; the input gradient matches on every column < E and stores whole tiles
    at n >= E as 0. The trimmed GEMMs get F with NaN in the empty chunks (the stack's hop leaves
    them unwritten): they must never read them — d = 153 puts E = 306 inside a 16-byte vector of
    the 16-byte-staged path."""
    n, h = 1500, 3
    K = d * (h + 1)
    counts = torch.zeros(h * n, dtype=torch.int32)
    for j, ne in enumerate(nonempty):
        if ne:
            counts[j * n:(j + 1) * n:7] = 2
    rowptr = torch.cat([torch.zeros(1, dtype=torch.int32), counts.cumsum(0).to(torch.int32)]).to(DEV)
    c = max([j + 1 for j, ne in enumerate(nonempty) if ne], default=0)
    E = d * (1 + c)
    g = torch.Generator().manual_seed(5)
    F = torch.randn(n, K, generator=g)
    F[:, E:] = 0
    Fnan = F.clone()
    Fnan[:, E:] = float("nan")
    zc = lambda dim: (rowptr, n, h, d, dim)  # noqa: E731
    W = torch.randn(2 * d, K, generator=g)
    full, _, _, ref, _ = _gemm(n, 2 * d, K, "NT", A=F, B=W)
    trim, _, _, _, _ = _gemm(n, 2 * d, K, "NT", A=Fnan, B=W, zc=zc(0))
    assert torch.equal(full, trim)
    assert (trim.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    dUG = torch.randn(n, 2 * d, generator=g)  # dF = dUG W
    full, _, _, _, _ = _gemm(n, K, 2 * d, "NN", A=dUG, B=W)
    trim, _, _, _, _ = _gemm(n, K, 2 * d, "NN", A=dUG, B=W, zc=zc(1))
    assert torch.equal(full[:, :E], trim[:, :E])
    past = -(-E // 64) * 64  # past the tile (32 or 64 columns wide) that holds column E-1
    assert not trim[:, past:].any()
    dY = torch.randn(n, 2 * d, generator=g)  # dW = dY^T F (+ bias column)
    full, fcol, _, ref, _ = _gemm(2 * d, K, n, "TN", A=dY, B=F, ones=True)
    trim, tcol, _, _, _ = _gemm(2 * d, K, n, "TN", A=dY, B=Fnan, ones=True, zc=zc(1))
    assert torch.equal(full, trim) and torch.equal(fcol, tcol)
    assert not trim[:, E:].any()


@pytest.mark.parametrize("splits", [1, 3, 64])
def test_gemm_weight_grad_forced_splits(splits):
    """The weight-gradient kernel (A m-contiguous, B n-contiguous, long K) at forced split counts,
    including one workgroup per tile and more splits than a slice can fill."""
    C, col, _, ref, Am = _gemm(76, 77, 4099, "TN", ones=True, splits=splits)
    assert (C.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    rs = Am.double().sum(1)
    assert (col.double() - rs).abs().max().item() / rs.abs().max().item() < 2e-6


@pytest.mark.parametrize("bb", ["auto", "64", "80"])
def test_wgrad_grouped_matches_fp64(bb):
    """aimx_wgrad_grouped over the stack's shapes (76 x 76 / 152 x 304 / c5's 307 x 307 and
    614 x 614 with the bias column, long K: the LDS-block kernel with the block edge its rule picks,
    or 64- or 80-wide blocks forced by the AIMX_WGRAD_BB option), a short-K FFN shape, K = 1 and odd
    widths (unaligned rows: the LDS kernel's dword loads), the c5 [Wi; Wg] product (614 x 615, K =
    10240) and a 512 x 384 one: dW = dY^T X and db = sum_k dY against fp64, deterministic, counters
    left at zero."""
    from aimx import _lib
    opts = {} if bb == "auto" else {"AIMX_WGRAD_BB": int(bb)}
    with _lib.options(**opts):
        _wgrad_grouped_case()


def _wgrad_grouped_case():
    from aimx import ops, _lib
    g = torch.Generator().manual_seed(11)
    shapes = [(76, 76, 9170, True), (152, 304, 9170, True), (76, 76, 4099, False), (256, 256, 520, True),
              (36, 36, 1, True), (38, 38, 777, True), (8, 12, 64, False),
              (153, 153, 5000, True), (77, 45, 2500, False), (160, 81, 2048, True),  # LDS path: dword loads
              (307, 307, 10240, True), (614, 614, 4096, True), (145, 301, 3001, False), (163, 150, 2048, True),
              (614, 614, 10240, True), (512, 384, 12000, False)]
    probs, refs = [], []
    for M, N, K, bias in shapes:
        dy = torch.randn(K, M, generator=g)
        x = torch.randn(K, N, generator=g)
        dw = torch.full((M, N), float("nan"), device=DEV)
        db = torch.full((M,), float("nan"), device=DEV) if bias else None
        probs.append((dy.to(DEV), x.to(DEV), dw, db))
        refs.append((dy.double().t() @ x.double(), dy.double().sum(0) if bias else None))
    ops.wgrad_grouped(probs)
    outs = [(p[2].clone(), None if p[3] is None else p[3].clone()) for p in probs]
    for (dw, db), (rw, rb) in zip(outs, refs):
        assert torch.isfinite(dw).all()
        assert (dw.cpu().double() - rw).abs().max().item() / rw.abs().max().item() < 2e-6
        if rb is not None:
            assert (db.cpu().double() - rb).abs().max().item() / rb.abs().max().item() < 2e-6
    ops.wgrad_grouped(probs)
    for p, (dw, db) in zip(probs, outs):
        assert torch.equal(p[2], dw) and (db is None or torch.equal(p[3], db))
    assert int(_lib.counters(DEV).abs().sum().item()) == 0


@pytest.mark.parametrize("fused", [True, False])
def test_gemm_ones_column_bias_grad_and_splitk(fused):
    C, col, _, ref, Am = _gemm(76, 304, 9170, "TN", ones=True, splits=24, fused_reduce=fused)
    assert (C.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    rs = Am.double().sum(1)
    assert (col.double() - rs).abs().max().item() / rs.abs().max().item() < 2e-6
    # deterministic: a second run is bitwise identical, and the counters were left at zero
    C2, col2, _, _, _ = _gemm(76, 304, 9170, "TN", ones=True, splits=24, fused_reduce=fused)
    assert torch.equal(C, C2) and torch.equal(col, col2)
    from aimx import _lib
    assert int(_lib.counters(DEV).abs().sum().item()) == 0


@pytest.mark.parametrize("act,fn", [(0, torch.relu), (1, lambda v: torch.nn.functional.leaky_relu(v, 0.01)),
                                    (2, torch.nn.functional.elu), (3, torch.nn.functional.gelu),
                                    (4, torch.nn.functional.silu)])
def test_gemm_activation_epilogue(act, fn):
    C, _, pre, ref, _ = _gemm(500, 76, 304, "NT", bias=True, act=act)
    assert (pre.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    assert (C.double() - fn(ref)).abs().max().item() / fn(ref).abs().max().item() < 2e-6


# --------------------------------------------------------------------------------------- layers
@pytest.mark.parametrize("n,width,xs,off", [(37, 256, 180, 0), (1031, 512, 359, 0), (19, 1024, 717, 1), (5, 8, 0, 0),
                                         (5, 8, 8, 3)])
def test_act_backward_two_sources(n, width, xs, off):
    """aimx_act_backward2 (the embedding projection's act' over the x_self / x_other gradients, one
    launch) equals dy * act'(pre) per element; dy0 a strided view (ld = width + off), dy1 contiguous."""
    from aimx import _lib
    lib = _lib.load()
    P = _lib.ptr
    g = torch.Generator(device="cpu").manual_seed(n + width)
    pre = torch.randn(n, width, generator=g).to(DEV)
    big = torch.randn(n, width + off + 3, generator=g).to(DEV)
    dy0 = big[:, off:off + xs]
    dy1 = torch.randn(n, width - xs, generator=g).to(DEV)
    out = torch.full((n, width), float("nan"), device=DEV)
    assert lib.aimx_act_backward2(_lib.ACT_KIND["silu"], P(dy0), big.stride(0), xs, P(dy1), max(1, width - xs), P(pre),
                                  width, n, width, P(out), width, _lib.stream_ptr(pre.device)) == 0
    p64 = pre.double()
    sg = torch.sigmoid(p64)
    ref = torch.cat([dy0.double(), dy1.double()], 1) * (sg * (1 + p64 * (1 - sg)))
    assert torch.allclose(out.double(), ref, rtol=1e-6, atol=1e-6)


def test_shell_layer_standalone():
    from models.layers import ShellConvolutionLayer
    z = load_golden("mp_general")
    layer = ShellConvolutionLayer(38, 38, num_hops=3)
    layer.load_state_dict({k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param.")})
    layer = layer.to(DEV).eval()
    x = torch.from_numpy(z["x"]).to(DEV).requires_grad_()
    y = layer(x, torch.from_numpy(z["tgt"]).to(DEV), torch.from_numpy(z["src"]).to(DEV))
    (y * torch.from_numpy(z["w"]).to(DEV)).sum().backward()
    ours = {"y": y.detach().cpu().numpy(), "grad_x": x.grad.cpu().numpy()}
    for k, p in layer.named_parameters():
        ours["grad." + k] = p.grad.cpu().numpy()
    ref = {k: z[k] for k in ours}
    bad = parity_failures(ours, None, ref)
    assert not bad, bad


@pytest.mark.parametrize("tag", ["sq_nm0", "noproj", "noproj_nm0", "rect", "rect_nm3"])
def test_shell_layer_contract(tag):
    """The general ShellConvolutionLayer contract against reference-generated fixtures
    (shell_layers.npz, tests/golden/make_golden.py case_shell): no MLP blocks (cli.py:106-107),
    no global_skip_proj (input_dim == output_dim: global_skip = x.clone(), layers.py:61,86-89),
    output_dim != atom_input_dim, hop-offset and plain targets; outputs and every gradient vs the
    fp64 oracle, the fixture's fp32 error as the floor once the fp32 oracle pins it."""
    from models.layers import ShellConvolutionLayer
    from test_oracle_golden import shell_layer_oracle
    z = load_golden("shell_layers")
    d, dout, h, nm = (int(v) for v in z[f"{tag}.dims"])
    layer = ShellConvolutionLayer(d, dout, num_hops=h, num_mlp_layers=nm)
    pre = f"{tag}.param."
    layer.load_state_dict({k[len(pre):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre)})
    layer = layer.to(DEV).eval()
    assert (layer.global_skip_proj is None) == tag.startswith("noproj")
    x = torch.from_numpy(z[f"{tag}.x"]).to(DEV).requires_grad_()
    y = layer(x, torch.from_numpy(z[f"{tag}.tgt"]).to(DEV), torch.from_numpy(z[f"{tag}.src"]).to(DEV))
    (y * torch.from_numpy(z[f"{tag}.w"]).to(DEV)).sum().backward()
    ours = {"y": y.detach().cpu().numpy(), "grad_x": x.grad.cpu().numpy()}
    ours.update({"grad." + k: p.grad.cpu().numpy() for k, p in layer.named_parameters()})
    torch.set_num_threads(8)
    o32 = shell_layer_oracle(z, tag, torch.float32)
    o64 = shell_layer_oracle(z, tag, torch.float64)
    assert set(ours) == set(o64), set(ours) ^ set(o64)
    bad = parity_failures(ours, {k: z[f"{tag}.{k}"] for k in ours}, o64, oracle32=o32)
    assert not bad, bad


def test_attention_pool_standalone():
    from models.pooling import MultiHeadAttentionPoolingLayer
    _, om = _oracle()
    z = load_golden("attn_pool")
    params = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param.")}
    pool = MultiHeadAttentionPoolingLayer(64, num_heads=4, initial_temperature=0.7)
    pool.load_state_dict(params)
    pool = pool.to(DEV)
    x = torch.from_numpy(z["x"]).to(DEV).requires_grad_()
    pooled, attn = pool(x, torch.from_numpy(z["batch"]).to(DEV))
    ((pooled * torch.from_numpy(z["wp"]).to(DEV)).sum() + (attn * torch.from_numpy(z["wa"]).to(DEV)).sum()).backward()
    ours = {"pooled": pooled.detach().cpu().numpy(), "attn": attn.detach().cpu().numpy(),
            "grad_x": x.grad.cpu().numpy()}
    for k, p in pool.named_parameters():
        ours["grad." + k] = p.grad.cpu().numpy()
    # fp64 oracle of the same layer
    p64 = {"pool." + k: v.double().requires_grad_() for k, v in params.items()}
    x64 = torch.from_numpy(z["x"]).double().requires_grad_()
    b = torch.from_numpy(z["batch"])
    pp, aa = om.attention_pool(p64, "pool.", x64, b, 4, int(b.max()) + 1)
    ((pp * torch.from_numpy(z["wp"]).double()).sum() + (aa * torch.from_numpy(z["wa"]).double()).sum()).backward()
    ref64 = {"pooled": pp.detach().numpy(), "attn": aa.detach().numpy(), "grad_x": x64.grad.numpy()}
    ref64.update({"grad." + k[5:]: v.grad.numpy() for k, v in p64.items()})
    p32 = {"pool." + k: v.clone().requires_grad_() for k, v in params.items()}
    x32 = torch.from_numpy(z["x"]).requires_grad_()
    pp, aa = om.attention_pool(p32, "pool.", x32, b, 4, int(b.max()) + 1)
    ((pp * torch.from_numpy(z["wp"])).sum() + (aa * torch.from_numpy(z["wa"])).sum()).backward()
    o32 = {"pooled": pp.detach().numpy(), "attn": aa.detach().numpy(), "grad_x": x32.grad.numpy()}
    o32.update({"grad." + k[5:]: v.grad.numpy() for k, v in p32.items()})
    bad = parity_failures(ours, {k: z[k] for k in ours}, ref64, oracle32=o32)
    assert not bad, bad


@pytest.mark.parametrize("C,H,strided", [(128, 4, False), (256, 4, True), (256, 1, False), (300, 3, False),
                                           (512, 4, False), (512, 8, True), (1024, 4, False), (1024, 8, False),
                                           (76, 4, False), (1100, 2, False)])
def test_attention_pool_shapes(C, H, strided):
    """Row-resident path (one chunk, several chunks), general path (odd widths, > 128 atoms, > 512
    atoms: global scratch), strided x, 1..8 heads, an upstream attention gradient, and features
    with a large common mean (the softmax-backward cancellation case) vs the fp64 oracle."""
    from models.pooling import MultiHeadAttentionPoolingLayer
    _, om = _oracle()
    g = torch.Generator().manual_seed(C * 10 + H)
    sizes = [1, 2, 7, 18, 29, 31, 32, 33, 40, 47, 48, 49, 64, 65, 100, 128, 129, 300, 600, 3]
    batch = torch.cat([torch.full((s,), i, dtype=torch.long) for i, s in enumerate(sizes)])
    n = batch.numel()
    x = 3.0 + torch.randn(n, C + (4 if strided else 0), generator=g)
    pool = MultiHeadAttentionPoolingLayer(C, num_heads=H, initial_temperature=0.7)
    with torch.no_grad():
        for lin in pool.attention_weights:
            lin.weight.copy_(torch.randn(1, C, generator=g) * 0.1)
            lin.bias.copy_(torch.randn(1, generator=g))
    params = {k: v.detach().clone() for k, v in pool.state_dict().items()}
    wp = torch.randn(len(sizes), C, generator=g)
    wa = torch.randn(H, n, generator=g)
    pool = pool.to(DEV)
    xd = x.to(DEV)[:, :C].requires_grad_() if not strided else x.to(DEV).requires_grad_()
    xin = xd[:, :C] if strided else xd
    pooled, attn = pool(xin, batch.to(DEV))
    ((pooled * wp.to(DEV)).sum() + (attn * wa.to(DEV)).sum()).backward()
    ours = {"pooled": pooled.detach().cpu().numpy(), "attn": attn.detach().cpu().numpy(),
            "grad_x": xd.grad[:, :C].cpu().numpy()}
    for k, p in pool.named_parameters():
        ours["grad." + k] = p.grad.cpu().numpy()
    refs = {}
    for dt in (torch.float32, torch.float64):  # the reference's fp32 algorithm (its noise floor) and fp64
        pd = {"pool." + k: v.detach().to(dt).requires_grad_() for k, v in params.items()}
        xr = x[:, :C].detach().to(dt).requires_grad_()
        pp, aa = om.attention_pool(pd, "pool.", xr, batch, H, len(sizes))
        ((pp * wp.to(dt)).sum() + (aa * wa.to(dt)).sum()).backward()
        ref = {"pooled": pp.detach().numpy(), "attn": aa.detach().numpy(), "grad_x": xr.grad.numpy()}
        ref.update({"grad." + k[5:]: v.grad.numpy() for k, v in pd.items()})
        refs[dt] = ref
    bad = parity_failures(ours, None, refs[torch.float64], oracle32=refs[torch.float32])
    assert not bad, bad


# ----------------------------------------------------------------------------------- full model
def _build_model(cfg, seed):
    from models import GNN
    _, om = _oracle()
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    m = GNN(fs, cfg["hidden_dim"], cfg["output_dim"], num_shells=cfg["num_shells"],
            num_message_passing_layers=cfg["num_message_passing_layers"], ffn_num_layers=cfg["ffn_num_layers"],
            pooling_type=cfg["pooling_type"], embedding_dim=cfg["embedding_dim"],
            use_partial_charges=cfg["use_partial_charges"], activation_type=cfg["activation"],
            shell_conv_num_mlp_layers=cfg["shell_conv_num_mlp_layers"], attention_num_heads=cfg["attention_num_heads"],
            loss_function=cfg["loss_function"], use_stereochemistry=cfg.get("use_stereochemistry", False))
    m.load_state_dict(om.seeded_params(cfg, seed))
    return m.to(DEV).eval()


def _oracle_run(z, cfg, inputs, dtype):
    _, om = _oracle()
    af, edges, batch, tc = inputs
    p = {k: v.to(dtype).requires_grad_() for k, v in om.seeded_params(cfg, int(z["seed"])).items()}
    tet, cis, trans = case_stereo(z)
    out, attn, q = om.gnn_forward(p, cfg, af, edges, batch, tc.to(dtype), tet=tet, cis=cis, trans=trans)
    (out * torch.from_numpy(z["loss_w"]).to(dtype)).sum().backward()
    res = {"out": out.detach().numpy()}
    if attn is not None:
        res["attn"] = attn.detach().numpy()
    if q is not None:
        res["q"] = q.detach().numpy()
    for k, v in p.items():
        if v.grad is not None:
            res["grad." + k] = v.grad.numpy()
    return add_sketches(res, z)


# config-sized batches (BASELINE configs[3] / [4] per GPU): the c4s / c5s architectures and seeds on
# 512 / 256 synthetic 40-atom molecules (the bench's synth40 source), every output and gradient
# compared element-wise with the fp64 oracle (no sketches)
FULL_SIZE = {"c4": ("c4s", 512), "c5": ("c5s", 256)}


def full_size_case(name):
    """(fixture of the architecture, cfg, CPU inputs, loss weights) of a config-sized case."""
    from aimx import data as adata
    from aimx.synth import synth_molecules
    base, mols = FULL_SIZE[name]
    z = load_golden(base)
    cfg = dict(load_case(base)[1])
    col = adata.collate(synth_molecules(mols, seed=1000 + mols), cfg["num_shells"])
    from golden_cases import FEATURE_KEYS
    feats = torch.from_numpy(col["feats"].astype(np.int64))
    af = {k: feats[:, i].contiguous() for i, k in enumerate(FEATURE_KEYS)}
    inputs = (af, torch.from_numpy(col["edges"].astype(np.int64)).reshape(-1, 2),
              torch.from_numpy(col["batch"].astype(np.int64)), torch.zeros(mols))
    loss_w = np.random.default_rng(mols).standard_normal((mols, cfg["output_dim"])).astype(np.float32)
    return z, cfg, inputs, loss_w


def _run_full(cfg, seed, inputs, loss_w, device, dtype=torch.float32):
    """(outputs and parameter gradients) of loss = sum(out * loss_w): the GPU model (device 'cuda')
    or the oracle (device 'cpu', dtype fp32 / fp64)."""
    af, edges, batch, tc = inputs
    e0 = torch.empty(0, 2, dtype=torch.long)
    if device == "cpu":
        _, om = _oracle()
        p = {k: v.to(dtype).requires_grad_() for k, v in om.seeded_params(cfg, seed).items()}
        cap = {}
        out, attn, _ = om.gnn_forward(p, cfg, af, edges, batch, tc.to(dtype), capture=cap)
        (out * torch.from_numpy(loss_w).to(dtype)).sum().backward()
        res = {"grad." + k: v.grad.numpy() for k, v in p.items() if v.grad is not None}
        if dtype == torch.float64 and "pool_scores" in cap:
            res["scale:grad.pooling.temperature"] = om.temperature_scale(cap)
    else:
        model = _build_model(cfg, seed)
        d = lambda t: t.to(DEV)  # noqa: E731
        out, attn, _ = model({k: d(v) for k, v in af.items()}, d(edges), d(batch), d(tc),
                             torch.empty(0, 4, dtype=torch.long, device=DEV), d(e0), d(e0))
        (out * torch.from_numpy(loss_w).to(DEV)).sum().backward()
        res = {"grad." + k: p.grad.cpu().numpy() for k, p in model.named_parameters() if p.grad is not None}
    res["out"] = out.detach().cpu().numpy()
    res["attn"] = attn.detach().cpu().numpy()
    return res


@pytest.mark.parametrize("name", sorted(FULL_SIZE))
def test_model_full_size(name):
    """c4 / c5 at their configured per-GPU batch (512 x 40-atom molecules h512 3 hops; 256 x
    40-atom h1024 6 hops): outputs, attention and every parameter gradient, element for element,
    within the parity contract against the fp64 oracle (the floor: the larger error of the oracle's
    fp32 run on the batch and on the molecule-reversed batch — the reference's ATen ops, pinned by
    tests/test_oracle_golden.py — golden_cases.reversed_molecules). Exercises what the 64 / 32-molecule
    fixtures cannot: the weight-streamed MLP at its 96 / 48-row chunks, full-K (~20 k atom) split-K
    weight gradients, multi-window hop tiling."""
    z, cfg, inputs, loss_w = full_size_case(name)
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    seed = int(z["seed"])
    ref64 = _run_full(cfg, seed, inputs, loss_w, "cpu", torch.float64)
    ref32 = _run_full(cfg, seed, inputs, loss_w, "cpu", torch.float32)
    rin, rlw, unperm = reversed_molecules(inputs, loss_w)
    ref32r = unperm(_run_full(cfg, seed, rin, rlw, "cpu", torch.float32))
    ours = _run_full(cfg, seed, inputs, loss_w, "cuda")
    assert set(ours) == {k for k in ref64 if not k.startswith("scale:")}
    bad = parity_failures(ours, None, ref64, oracle32=[ref32, ref32r])
    assert not bad, bad


@pytest.mark.parametrize("name", CASES)
def test_model_case(name):
    z, cfg, inputs = load_case(name)
    torch.set_num_threads(8)
    ref64 = _oracle_run(z, cfg, inputs, torch.float64)
    ref32 = fixture_refs(z)
    must = set(ref32)
    # the oracle's fp32 run on the same inputs: it must pin the fixture (conftest.pin_tol) before
    # the fixture's own fp32 error becomes the floor; for tensors the fixture did not store it is
    # the floor itself (the reference's ATen ops, pinned by tests/test_oracle_golden.py)
    oracle32 = _oracle_run(z, cfg, inputs, torch.float32)
    model = _build_model(cfg, int(z["seed"]))
    af, edges, batch, tc = load_case(name, DEV)[2]
    out, attn, q = model(af, edges, batch, tc, *case_stereo(z, DEV))
    (out * torch.from_numpy(z["loss_w"]).to(DEV)).sum().backward()
    ours = {"out": out.detach().cpu().numpy()}
    if attn is not None:
        ours["attn"] = attn.detach().cpu().numpy()
    if q is not None:
        ours["q"] = q.detach().cpu().numpy()
    for k, p in model.named_parameters():
        if p.grad is not None:
            ours["grad." + k] = p.grad.cpu().numpy()
    add_sketches(ours, z)
    # every gradient the reference produced must be produced here too
    for k in must:
        assert k in ours, k
    bad = parity_failures(ours, ref32, ref64, oracle32=oracle32)
    assert not bad, bad


def test_forward_hooks_fire():
    z, cfg, _ = load_case("c1")
    model = _build_model(cfg, int(z["seed"]))
    seen = {}
    model.pooling.register_forward_hook(lambda m, a, o: seen.__setitem__("pool", o[0].shape))
    model.concat_self_other.register_forward_hook(lambda m, a, o: seen.__setitem__("cat", o.shape))
    af, edges, batch, tc = load_case("c1", DEV)[2]
    e0 = torch.empty(0, 2, dtype=torch.long, device=DEV)
    with torch.no_grad():
        model(af, edges, batch, tc, torch.empty(0, 4, dtype=torch.long, device=DEV), e0, e0)
    assert seen["pool"] == (32, cfg["hidden_dim"]) and seen["cat"][0] == z["feats"].shape[0]


def test_train_mode_dropout_statistics_and_determinism():
    """Dropout (p=0.05) in the fused epilogue: ~5% of block activations dropped; a fixed seed gives
    identical results; eval mode is deterministic and dropout-free."""
    from aimx import ops
    from aimx.plan import GraphPlan
    z, cfg, _ = load_case("c2")
    model = _build_model(cfg, int(z["seed"]))
    af, edges, batch, tc = load_case("c2", DEV)[2]
    layers = model.message_passing_layers
    params = []
    for l in layers:
        params += l._aimx_params()
    n, d = z["feats"].shape[0], cfg["x_other_dim"]
    x = torch.randn(n, d, device=DEV)
    plan = GraphPlan(n, 3, edges=edges, batch=batch, num_graphs=512)
    seed = torch.tensor([1234], device=DEV)
    kw = dict(num_hops=3, num_layers=3, num_mlp=2, act="silu", training=True, drop_p=0.05, drop_seed=seed)
    y1 = ops.message_passing_stack(plan, x, params, **kw)
    y2 = ops.message_passing_stack(plan, x, params, **kw)
    assert torch.equal(y1, y2)
    y3 = ops.message_passing_stack(plan, x, params, **dict(kw, drop_seed=torch.tensor([99], device=DEV)))
    assert not torch.equal(y1, y3)
    y0 = ops.message_passing_stack(plan, x, params, **dict(kw, training=False))
    assert not torch.equal(y0, y1)


# ------------------------------------------------------------------------------------ optimizer
@pytest.mark.parametrize("max_norm,wd", [(1.0, 0.0), (None, 0.0), (0.05, 0.01)])
def test_fused_adam_matches_torch_clip_and_adam(max_norm, wd):
    """aimx_fused_adam == clip_grad_norm_(max_norm) + torch.optim.Adam (trainer.py:163-164, 221-223),
    two parameter groups with different lr, several steps (fp32 rounding only)."""
    from aimx.optim import FusedAdam
    g = torch.Generator().manual_seed(7)
    shapes = [(76, 304), (152,), (256, 256), (3,), (70000,)]
    p0 = [torch.randn(s, generator=g) for s in shapes]
    ours = [x.clone().to(DEV).requires_grad_() for x in p0]
    ref = [x.clone().to(DEV).requires_grad_() for x in p0]
    groups = lambda ps: [{"params": ps[:3], "lr": 1e-3}, {"params": ps[3:], "lr": 3e-4}]  # noqa: E731
    opt = FusedAdam(groups(ours), weight_decay=wd, max_grad_norm=max_norm)
    topt = torch.optim.Adam(groups(ref), weight_decay=wd)
    for step in range(5):
        grads = [torch.randn(s, generator=g) * (0.01 + step) for s in shapes]
        for a, b, gr in zip(ours, ref, grads):
            a.grad = gr.to(DEV).clone()
            b.grad = gr.to(DEV).clone()
        opt.step()
        if max_norm:
            tn = torch.nn.utils.clip_grad_norm_(ref, max_norm)
            assert abs(float(opt.last_grad_norm) - float(tn)) <= 1e-5 * float(tn)
        topt.step()
        for a, b in zip(ours, ref):
            assert torch.allclose(a.grad, b.grad, rtol=1e-6, atol=1e-9)
    for a, b in zip(ours, ref):
        assert norm_rel(a.detach().cpu().numpy(), b.detach().cpu().numpy()) < 1e-6
        st_a, st_b = opt.state[a], topt.state[b]
        assert norm_rel(st_a["exp_avg"].cpu().numpy(), st_b["exp_avg"].cpu().numpy()) < 1e-6
        assert norm_rel(st_a["exp_avg_sq"].cpu().numpy(), st_b["exp_avg_sq"].cpu().numpy()) < 1e-6
        assert float(st_a["step"]) == float(st_b["step"]) == 5.0


def test_fused_adam_missing_gradients_keep_per_parameter_steps():
    """Steps where some parameters have no gradient (e.g. a batch without edges skips message
    passing, gnn.py:287): torch.optim.Adam advances only the stepped parameters' state['step'];
    the fused step must too (per-parameter bias corrections)."""
    from aimx.optim import FusedAdam
    g = torch.Generator().manual_seed(11)
    shapes = [(64, 32), (32,), (1000,), (5,)]
    p0 = [torch.randn(s, generator=g) for s in shapes]
    ours = [x.clone().to(DEV).requires_grad_() for x in p0]
    ref = [x.clone().to(DEV).requires_grad_() for x in p0]
    opt = FusedAdam(ours, lr=1e-2, max_grad_norm=1.0)
    topt = torch.optim.Adam(ref, lr=1e-2)
    present = [[0, 1, 2, 3], [0, 2], [1, 3], [0, 1, 2, 3], [2], [0, 1, 2, 3]]
    for have in present:
        for i, (a, b) in enumerate(zip(ours, ref)):
            if i in have:
                gr = torch.randn(shapes[i], generator=g)
                a.grad, b.grad = gr.to(DEV).clone(), gr.to(DEV).clone()
            else:
                a.grad = b.grad = None
        opt.step()
        torch.nn.utils.clip_grad_norm_([b for b in ref if b.grad is not None], 1.0)
        topt.step()
    for a, b in zip(ours, ref):
        assert float(opt.state[a]["step"]) == float(topt.state[b]["step"])
        assert norm_rel(a.detach().cpu().numpy(), b.detach().cpu().numpy()) < 1e-6
        assert norm_rel(opt.state[a]["exp_avg_sq"].cpu().numpy(), topt.state[b]["exp_avg_sq"].cpu().numpy()) < 1e-6


def test_fused_adam_add_param_group_after_steps():
    """optimizer.add_param_group() after the first step (torch.optim.Adam supports it): the step
    counters and learning rates grow with the groups; existing parameters keep their counts."""
    from aimx.optim import FusedAdam
    g = torch.Generator().manual_seed(13)
    shapes1, shapes2 = [(40, 8), (8,)], [(300,), (7, 3)]
    p1 = [torch.randn(s, generator=g) for s in shapes1]
    p2 = [torch.randn(s, generator=g) for s in shapes2]
    ours1, ref1 = [x.clone().to(DEV).requires_grad_() for x in p1], [x.clone().to(DEV).requires_grad_() for x in p1]
    ours2, ref2 = [x.clone().to(DEV).requires_grad_() for x in p2], [x.clone().to(DEV).requires_grad_() for x in p2]
    opt = FusedAdam(ours1, lr=1e-2, max_grad_norm=1.0)
    topt = torch.optim.Adam(ref1, lr=1e-2)

    def step(ours, ref):
        for a, b in zip(ours, ref):
            gr = torch.randn(a.shape, generator=g)
            a.grad, b.grad = gr.to(DEV).clone(), gr.to(DEV).clone()
        opt.step()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        topt.step()
    for _ in range(3):
        step(ours1, ref1)
    opt.add_param_group({"params": ours2, "lr": 3e-3})
    topt.add_param_group({"params": ref2, "lr": 3e-3})
    for _ in range(2):
        step(ours1 + ours2, ref1 + ref2)
    for a, b in zip(ours1 + ours2, ref1 + ref2):
        assert float(opt.state[a]["step"]) == float(topt.state[b]["step"])
        assert norm_rel(a.detach().cpu().numpy(), b.detach().cpu().numpy()) < 1e-6


def test_hop_segment_aligned_tiles_bit_exact():
    """Molecule ids (row_seg) only move the hop's tile cuts: forward and backward are bit-identical
    with and without them, on a large multi-molecule graph (thousands of tiles, cuts both aligned
    and not: one 200-atom molecule exceeds the 64-row alignment window)."""
    from aimx.plan import GraphPlan
    from aimx import ops
    _, om = _oracle()
    z = load_golden("c2")
    e0 = torch.from_numpy(z["edges"].astype(np.int64))
    b0 = torch.from_numpy(z["batch"].astype(np.int64)) if "batch" in z.files else None
    n0 = z["feats"].shape[0]
    if b0 is None:
        pytest.skip("fixture has no batch")
    reps = 6
    e = torch.cat([e0 + r * n0 for r in range(reps)], 0)
    g0 = int(b0.max()) + 1
    b = torch.cat([b0 + r * g0 for r in range(reps)], 0)
    # one long molecule: merge 12 consecutive molecules' ids (edges stay inside it)
    b = torch.where((b >= 100) & (b < 112), torch.full_like(b, 100), b)
    n = n0 * reps
    x = torch.randn(n, 76, generator=torch.Generator().manual_seed(9))
    ref = torch.cat(om.message_passing(x, e[:, 0], e[:, 1], 3), 0)
    outs, grads = [], []
    w = torch.randn(ref.shape, generator=torch.Generator().manual_seed(10)).to(DEV)
    for batch in (None, b.to(DEV)):
        plan = GraphPlan(n, 3, edges=e.to(DEV), batch=batch, num_graphs=None if batch is None else int(b.max()) + 1)
        xg = x.to(DEV).requires_grad_()
        out = ops.hop(plan, xg)
        (out * w).sum().backward()
        outs.append(out.detach().cpu())
        grads.append(xg.grad.cpu())
    assert torch.equal(outs[0], ref) and torch.equal(outs[1], ref)
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("rows,cols,weighted", [(520, 1, False), (512, 12, False), (512, 12, True), (3, 5, True)])
def test_l1_losses_match_reference_criteria(rows, cols, weighted):
    """models.L1Loss == nn.L1Loss and models.WeightedL1Loss == the reference's WeightedL1Loss
    (losses.py:14-48: sum over tasks of w |p - y|, mean over samples): values and gradients,
    including exact ties (sign(0) = 0)."""
    from models import L1Loss, WeightedL1Loss
    g = torch.Generator().manual_seed(rows + cols)
    p = torch.randn(rows, cols, generator=g)
    y = torch.randn(rows, cols, generator=g)
    y[0, 0] = p[0, 0]  # a tie
    w = torch.rand(cols, generator=g) + 0.5
    pg = p.to(DEV).requires_grad_()
    crit = WeightedL1Loss(w).to(DEV) if weighted else L1Loss()
    loss = crit(pg, y.to(DEV))
    loss.backward()
    p64 = p.double().requires_grad_()
    ref = ((p64 - y.double()).abs() * w.double()).sum(1).mean() if weighted else (p64 - y.double()).abs().mean()
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-6 * max(1.0, abs(ref.item()))
    assert (pg.grad.cpu().double() - p64.grad).abs().max().item() <= 1e-7
    assert pg.grad[0, 0].item() == 0.0


@pytest.mark.parametrize("weighted", [False, True])
def test_l1_loss_rows_of_padded_prediction(weighted):
    """ops.l1_loss(pred, target, rows=B) on a padded [B + 8, T] prediction (the captured train
    step's static batch) == the loss of pred[:B] through autograd's slice: bit-identical value and
    gradient, padding rows' gradient exactly 0 (they start as NaN in the buffer)."""
    from aimx import ops
    g = torch.Generator().manual_seed(5)
    B, T = 512, 12
    p = torch.randn(B + 8, T, generator=g).to(DEV)
    y = torch.randn(B, T, generator=g).to(DEV)
    w = (torch.rand(T, generator=g) + 0.5).to(DEV) if weighted else None
    a = p.clone().requires_grad_()
    la = ops.l1_loss(a, y, weights=w, per_sample=weighted, rows=B)
    la.backward()
    b = p.clone().requires_grad_()
    lb = ops.l1_loss(b[:B], y, weights=w, per_sample=weighted)
    lb.backward()
    assert torch.equal(la, lb)
    assert torch.equal(a.grad, b.grad)
    assert torch.equal(a.grad[B:], torch.zeros(8, T, device=DEV))


def test_l1_loss_accum_bookkeeping():
    """ops.l1_loss(..., accum=...) == the captured step's former torch bookkeeping
    (loss_sum.add_(loss * B), nan_count.add_(isnan(pred[:B]).any()), steps.add_(1)): bit-identical
    loss sums over several steps, NaN rows counted only inside the loss rows."""
    from aimx import ops
    g = torch.Generator().manual_seed(9)
    B, T = 512, 3
    ls, nc, st = (torch.zeros((), device=DEV), torch.zeros((), dtype=torch.int32, device=DEV),
                  torch.zeros((), dtype=torch.int64, device=DEV))
    ref_ls, ref_nc = torch.zeros((), device=DEV), torch.zeros((), dtype=torch.int32, device=DEV)
    for k in range(5):
        p = torch.randn(B + 8, T, generator=g).to(DEV)
        y = torch.randn(B, T, generator=g).to(DEV)
        if k == 2:
            p[7, 1] = float("nan")  # inside the loss rows: counted
        if k == 3:
            p[B + 2, 0] = float("nan")  # a padding row: not counted (not an output of the batch)
        loss = ops.l1_loss(p, y, rows=B, accum=(ls, nc, st, float(B)))
        ref = ops.l1_loss(p, y, rows=B)
        assert torch.equal(loss, ref) or (torch.isnan(loss).item() and torch.isnan(ref).item())
        ref_ls.add_(ref.detach() * B)
        ref_nc.add_(torch.isnan(p[:B]).any().to(torch.int32))
    torch.testing.assert_close(ls, ref_ls, rtol=0, atol=0, equal_nan=True)
    assert int(nc.item()) == int(ref_nc.item()) == 1
    assert int(st.item()) == 5


@pytest.mark.parametrize("name", ["c1", "c2", "c3"])
def test_fused_head_matches_module_path(name, monkeypatch):
    """The fused post-pool head (one launch forward, one + a grouped weight-gradient launch
    backward) against the per-module path (post_pooling_projection -> ffn -> skip_transform ->
    output_layer on the fused GEMM ops): outputs and every gradient, eval mode."""
    z, cfg, _ = load_case(name)
    af, edges, batch, tc = load_case(name, DEV)[2]
    e_empty = torch.empty(0, 2, dtype=torch.long, device=DEV)
    w = torch.from_numpy(z["loss_w"]).to(DEV)
    res = []
    import models.gnn as mg
    for off in ("0", "1"):
        monkeypatch.setattr(mg, "FUSED_HEAD", off == "0")
        model = _build_model(cfg, int(z["seed"]))
        assert model._aimx_head_ok() == (off == "0")
        out, _, _ = model(af, edges, batch, tc, torch.empty(0, 4, dtype=torch.long, device=DEV), e_empty, e_empty)
        (out * w).sum().backward()
        g = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
        res.append((out.detach().clone(), g))
    (o1, g1), (o2, g2) = res
    assert norm_rel(o1.cpu().numpy(), o2.cpu().numpy()) < 1e-5
    assert g1.keys() == g2.keys()
    for k in g1:
        if "attention_weights" in k and k.endswith("bias"):
            continue  # exactly 0 in exact arithmetic (softmax shift invariance): both are ~1e-19 noise
        assert norm_rel(g1[k].cpu().numpy(), g2[k].cpu().numpy()) < 2e-5, k


@pytest.mark.parametrize("rows", [None, 200])
def test_c5_head_path_matches_tiles(rows):
    """c5 at its configured batch (256 molecules, F = 1024: outside the fused head kernels; its
    G x F x F chain on k_gemm_deep, 256 tiles) against the same model on the LDS-staged tiles
    (AIMX_GEMM_DEEP option 0): outputs and every gradient. With the chain restricted to the first
    `rows` molecules (_aimx_head_rows, what graph capture sets: padding molecules never reach the
    head) the outputs equal the unrestricted run's first rows, and both paths agree on the
    gradients of the loss over them."""
    from aimx import _lib
    z, cfg, (af, edges, batch, tc), loss_w = full_size_case("c5")
    e0 = torch.empty(0, 2, dtype=torch.long, device=DEV)
    d = lambda t: t.to(DEV)  # noqa: E731
    args = ({k: d(v) for k, v in af.items()}, d(edges), d(batch), d(tc), torch.empty(0, 4, dtype=torch.long, device=DEV),
            e0, e0)
    w = torch.from_numpy(loss_w).to(DEV)
    res = []
    for deep in (16, 0):
        with _lib.options(AIMX_GEMM_DEEP=deep):
            model = _build_model(cfg, int(z["seed"]))
            assert not model._aimx_head_ok()
            if rows is not None:
                model.__dict__["_aimx_head_rows"] = rows
            out, _, _ = model(*args)
            (out * w[:out.shape[0]]).sum().backward()
            g = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
            res.append((out.detach().clone(), g))
    (o1, g1), (o2, g2) = res
    if rows is not None:
        assert o1.shape[0] == rows
        with torch.no_grad():
            of, _, _ = _build_model(cfg, int(z["seed"]))(*args)
        assert norm_rel(o1.cpu().numpy(), of[:rows].cpu().numpy()) < 1e-5
    assert norm_rel(o1.cpu().numpy(), o2.cpu().numpy()) < 1e-5
    assert g1.keys() == g2.keys()
    for k in g1:
        if "attention_weights" in k and k.endswith("bias"):
            continue  # exactly 0 in exact arithmetic (softmax shift invariance)
        assert norm_rel(g1[k].cpu().numpy(), g2[k].cpu().numpy()) < 2e-5, k


def test_fused_head_dropout():
    """Train mode: ~p of the head's hidden units dropped, a fixed seed is deterministic, another
    seed differs, and the backward runs (finite gradients)."""
    from aimx import ops
    g = torch.Generator().manual_seed(0)
    F, G = 256, 300
    mk = lambda *s: (torch.randn(*s, generator=g) * 0.1).to(DEV).requires_grad_()  # noqa: E731
    x = mk(G, F)
    wp, bp = mk(F, F), mk(F)
    blocks = [(mk(F, F), mk(F), mk(F, F), mk(F)) for _ in range(3)]
    ws, bs, wo, bo = mk(F, F), mk(F), mk(3, 2 * F), mk(3)
    kw = dict(act="silu", drop_p=0.2, training=True, skips=[False, True, False])
    s1 = torch.tensor([7], device=DEV)
    y1 = ops.head(x, wp, bp, blocks, ws, bs, wo, bo, seed=s1, **kw)
    y2 = ops.head(x, wp, bp, blocks, ws, bs, wo, bo, seed=s1.clone(), **kw)
    y3 = ops.head(x, wp, bp, blocks, ws, bs, wo, bo, seed=torch.tensor([8], device=DEV), **kw)
    y0 = ops.head(x, wp, bp, blocks, ws, bs, wo, bo, **dict(kw, training=False))
    assert torch.equal(y1, y2) and not torch.equal(y1, y3) and not torch.equal(y0, y1)
    y1.sum().backward()
    assert all(torch.isfinite(t.grad).all() for t in [x, wp, bp, ws, bs, wo, bo] + [p for b in blocks for p in b])


def test_head8_row_tiles_agree():
    """The 8-molecule head (H_in == F) at G = 2100 runs 8-row tiles (G >= 2048), at G = 300 4-row
    tiles: the same 2100 molecules through both (the big batch whole, then in 300-molecule
    slices) give the same outputs and input gradients row for row (1e-6), and the same weight
    gradients summed over the slices (1e-5 norm-relative)."""
    from aimx import ops
    g = torch.Generator().manual_seed(8)
    F, G = 256, 2100
    base = [torch.randn(G, F, generator=g) * 0.1, torch.randn(F, F, generator=g) * 0.06,
            torch.randn(F, generator=g) * 0.1]
    for _ in range(2):
        base += [torch.randn(F, F, generator=g) * 0.06, torch.randn(F, generator=g) * 0.1,
                 torch.randn(F, F, generator=g) * 0.06, torch.randn(F, generator=g) * 0.1]
    base += [torch.randn(F, F, generator=g) * 0.06, torch.randn(F, generator=g) * 0.1,
             torch.randn(2, 2 * F, generator=g) * 0.05, torch.randn(2, generator=g) * 0.1]
    # positive loss weights: the weight-gradient sums over 2100 rows do not cancel, so the whole-
    # batch and sliced sums agree to fp32 summation order (~1e-6)
    wy = (0.5 + torch.rand(G, 2, generator=g)).to(DEV)
    res = []
    for step in (G, 300):
        t = [b.to(DEV).requires_grad_() for b in base]
        ys = []
        for r0 in range(0, G, step):
            x = t[0][r0:r0 + step]
            y = ops.head(x, t[1], t[2], [tuple(t[3 + 4 * i:7 + 4 * i]) for i in range(2)], *t[11:15], act="silu",
                         skips=[False, True])
            (y * wy[r0:r0 + step]).sum().backward()
            ys.append(y.detach())
        torch.cuda.synchronize()
        res.append((torch.cat(ys), [q.grad.detach().clone() for q in t]))
    (y8, g8), (y4, g4) = res
    assert norm_rel(y8.cpu().numpy(), y4.cpu().numpy()) < 1e-6
    for i, (a, b) in enumerate(zip(g8, g4)):
        tol = 1e-6 if i == 0 else 1e-5  # [0]: the input gradient, row-local
        assert norm_rel(a.cpu().numpy(), b.cpu().numpy()) < tol, (i, norm_rel(a.cpu().numpy(), b.cpu().numpy()))


@pytest.mark.parametrize("G", [5, 300, 2100])
def test_fused_head_clusters_bit_identical(G, monkeypatch):
    """Clustered head launches (2, 4 or 8 workgroups per 16-molecule tile exchanging activations
    through HBM inside the launch; 2100 molecules = 132 tiles make the clusters loop over tiles)
    give bit-identical outputs and gradients to the one-workgroup-per-tile launch, with dropout,
    and never set the timeout word."""
    from aimx import _lib, ops
    g = torch.Generator().manual_seed(G)
    F, Hin = 256, 512
    base = [torch.randn(G, Hin, generator=g) * 0.1, torch.randn(F, Hin, generator=g) * 0.05,
            torch.randn(F, generator=g) * 0.1]
    for _ in range(2):
        base += [torch.randn(F, F, generator=g) * 0.06, torch.randn(F, generator=g) * 0.1,
                 torch.randn(F, F, generator=g) * 0.06, torch.randn(F, generator=g) * 0.1]
    base += [torch.randn(F, F, generator=g) * 0.06, torch.randn(F, generator=g) * 0.1,
             torch.randn(2, 2 * F, generator=g) * 0.05, torch.randn(2, generator=g) * 0.1]
    seed = torch.tensor([11], device=DEV)
    res = {}
    for S in ("1", "2", "4", "8"):
        monkeypatch.setattr(_lib, "HEAD_CLUSTER_FORCE", int(S))
        t = [b.to(DEV).requires_grad_() for b in base]
        x, wp, bp = t[:3]
        blocks = [tuple(t[3 + 4 * i:7 + 4 * i]) for i in range(2)]
        ws, bs, wo, bo = t[11:15]
        y = ops.head(x, wp, bp, blocks, ws, bs, wo, bo, act="silu", drop_p=0.1, training=True, seed=seed,
                     skips=[False, True])
        (y * torch.linspace(-1, 1, 2 * G, device=DEV).view(G, 2)).sum().backward()
        torch.cuda.synchronize()
        res[S] = [y.detach()] + [p.grad.detach() for p in t]
    assert int(_lib.head_sync(DEV)[0]) == 0, "a cluster wait timed out"
    assert int(_lib.head_sync(DEV)[1:].abs().sum()) == 0, "sync words not reset"
    for S in ("2", "4", "8"):
        for i, (a, b) in enumerate(zip(res["1"], res[S])):
            assert torch.equal(a, b), (S, i, (a - b).abs().max().item())


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "act_gelu", "stereo"])
def test_streamed_mlp_forced_parity(name, monkeypatch):
    """The AIMX_MLPS = 1 option (the weight-streamed node-update chain, mlp.hip k_mlps_*, the default
    for D > 128) forced onto the small-D cases keeps the model within the parity contract."""
    from aimx import _lib
    with _lib.options(AIMX_MLPS=1):
        test_model_case(name)


@pytest.mark.parametrize("name", ["c4s", "c5s"])
def test_per_gemm_mlp_path_parity_wide(name, monkeypatch):
    """The AIMX_MLPS = 0 option (one GEMM per MLP linear) at D = 153 / 307 stays within the parity
    contract."""
    from aimx import _lib
    with _lib.options(AIMX_MLPS=0):
        test_model_case(name)


def _stack_case(hidden, hops, mols, seed=0):
    from aimx import data as adata
    from aimx.plan import GraphPlan
    from aimx.synth import synth_molecules
    from models.layers import ShellConvolutionLayer
    torch.manual_seed(seed)
    col = adata.collate(synth_molecules(mols, seed=seed), hops)
    edges = torch.from_numpy(col["edges"]).to(DEV)
    batch = torch.from_numpy(col["batch"]).to(DEV)
    n, d = batch.shape[0], int(0.3 * hidden)
    plan = GraphPlan(n, hops, edges=edges, batch=batch, num_graphs=mols)
    layers = [ShellConvolutionLayer(d, d, num_hops=hops).to(DEV) for _ in range(3)]
    params = [p for l in layers for p in l._aimx_params()]
    return plan, params, n, d


@pytest.mark.parametrize("hidden,hops,mols,rt", [(512, 3, 512, None), (512, 3, 512, "1"), (1024, 6, 256, None),
                                                 (1024, 6, 256, "2"), (256, 3, 700, None), (640, 3, 64, None)])
def test_streamed_mlp_matches_per_gemm(hidden, hops, mols, rt, monkeypatch):
    """The weight-streamed chain against the per-GEMM path on the same stack, training mode with
    dropout: outputs and every gradient within 1e-5 norm-relative (both fp32, different summation
    order) — identical dropout masks are implied (one flipped mask element moves a tensor by far
    more). Config-sized batches (c4: 512 x 40-atom molecules, D = 153, 96-row chunks; c5: 256
    molecules, D = 307, two fragments per wave), forced small chunks (rt = 1 / 2: chunks > CUs, so
    workgroups loop over several), D = 76 forced onto the streamed kernel, and D = 192."""
    from aimx import ops
    plan, params, n, d = _stack_case(hidden, hops, mols)
    x = torch.randn(n, d, device=DEV)
    seed = torch.tensor([4321], device=DEV)
    kw = dict(num_hops=hops, num_layers=3, num_mlp=2, act="silu", training=True, drop_p=0.05, drop_seed=seed)
    w = torch.randn(n, d, device=DEV)
    res = {}
    from aimx import _lib
    for mode in ("0", "1"):
        opts = {"AIMX_MLPS": int(mode)}
        if rt is not None and mode == "1":
            opts["AIMX_MLPS_RT"] = int(rt)
        with _lib.options(**opts):
            xs = x.clone().requires_grad_()
            ps = [p.detach().clone().requires_grad_() for p in params]
            y = ops.message_passing_stack(plan, xs, ps, **kw)
            (y * w).sum().backward()
            torch.cuda.synchronize()
        res[mode] = [y.detach()] + [xs.grad] + [p.grad for p in ps]
    for i, (a, b) in enumerate(zip(res["1"], res["0"])):
        assert a is not None and b is not None, i
        assert torch.isfinite(a).all(), i
        err = norm_rel(a.cpu().numpy(), b.cpu().numpy())
        assert err < 1e-5, (i, err)


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "act_gelu", "stereo"])
def test_per_gemm_mlp_path_parity(name, monkeypatch):
    """The AIMX_MLPW = 0 option (one GEMM per MLP linear) keeps the small-D cases within the parity
    contract too (the default there is the weight-resident fused chain)."""
    from aimx import _lib
    with _lib.options(AIMX_MLPW=0):
        test_model_case(name)


# ------------------------------------------------------------------------------- stereochemistry
@pytest.mark.parametrize("D,M,with_ct", [(76, 40, True), (153, 7, True), (307, 0, True), (64, 25, False),
                                         (1024, 3, True)])
def test_stereo_features_match_oracle(D, M, with_ct):
    """ops.stereo_features ([x | cis/trans | tetrahedral], csrc/stereo.hip) against the oracle's
    restatement of gnn.py:376-497 run in fp64 with autograd: values and the input gradient,
    with atoms shared by several centres, a zero row (the normalize eps branch), no centres (the
    tetrahedral block is x itself) and no cis/trans items."""
    from aimx import ops
    _, om = _oracle()
    g = torch.Generator().manual_seed(D + M)
    n = 300
    x = torch.randn(n, D, generator=g)
    x[5] = 0.0
    tet = torch.randint(0, n, (M, 4), generator=g)
    if M:
        tet[0, 2] = 5  # a zero neighbour row
        tet[1] = tet[0]  # two centres naming the same atoms
    cis = torch.randint(0, n, (3, 2), generator=g) if with_ct else torch.empty(0, 2, dtype=torch.long)
    trans = torch.randint(0, n, (2, 2), generator=g) if with_ct else torch.empty(0, 2, dtype=torch.long)
    w = torch.randn(n, 3 * D, generator=g)
    xd = x.to(DEV).requires_grad_()
    out = ops.stereo_features(xd, tet.to(DEV), cis.to(DEV), trans.to(DEV))
    (out * w.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_()
    ref = torch.cat([x64, om.cis_trans(x64, cis, trans), om.tetrahedral(x64, tet)], -1)
    (ref * w.double()).sum().backward()
    assert norm_rel(out.detach().cpu().numpy(), ref.detach().numpy()) < 1e-6
    assert norm_rel(xd.grad.cpu().numpy(), x64.grad.numpy()) < 1e-5
