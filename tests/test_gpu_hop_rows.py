"""GPU parity of the odd-width / unaligned-row hop (csrc/hop_rows.hip) through the C ABI.

Reference op: ShellConvolutionLayer.message_passing, /root/reference/src/models/layers.py:133-167
(out[t] += x[src % N] in edge order, dim_size = num_hops * N) and its backward
(dx[j] += g[t] over edges with src % N == j, in edge order). The expected values are the
sequential fp32 sums (numpy ufunc.at runs in index order, like CPU scatter_add_ / index_put_), so
every check is bit-exact. Widths are the reference's D = int(0.3 * hidden) (gnn.py:100): 153 and
307, plus small odd ones; layouts are the standalone op's ([N, D] in, [h*N, D] out) and the
message-passing stack's (hop chunks written at column offset D of F = [x | chunks], the backward
reading F's hop chunks with the chunk-0 gradient and the outer residual fused, stack.hip).
"""
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


def _graph(kind, count, hops, seed=0):
    """(n, edges int64 [E, 2] (target, source), batch int64 [n]) of a collated batch."""
    from aimx import data as adata
    from aimx.synth import QM9Asset, synth_molecules
    if kind == "synth40":
        mols = synth_molecules(count, seed=seed)
    else:
        asset = QM9Asset()
        mols = asset.molecules(np.random.default_rng(seed).integers(0, len(asset), count))
    col = adata.collate(mols, hops)
    return col["batch"].shape[0], col["edges"].astype(np.int64), col["batch"].astype(np.int64)


def _fwd_ref(x, tgt, src, hops):
    n = x.shape[0]
    out = np.zeros((hops * n, x.shape[1]), np.float32)
    np.add.at(out, tgt, x[np.mod(src, n)])
    return out


def _bwd_ref(g, tgt, src, n):
    dx = np.zeros((n, g.shape[1]), np.float32)
    np.add.at(dx, np.mod(src, n), g[tgt])
    return dx


def _plan(n, hops, edges, batch):
    from aimx.plan import GraphPlan
    e = torch.from_numpy(edges).to(DEV)
    b = torch.from_numpy(batch).to(DEV) if batch is not None else None
    g = int(batch.max()) + 1 if batch is not None else None
    return GraphPlan(n, hops, edges=e, batch=b, num_graphs=g)


@pytest.mark.parametrize("kind,count,hops,d", [
    ("synth40", 64, 3, 153), ("synth40", 32, 6, 307), ("qm9", 256, 3, 38), ("qm9", 128, 4, 5),
    ("synth40", 48, 3, 2), ("qm9", 300, 3, 77)])
@pytest.mark.parametrize("with_batch", [True, False])
def test_hop_rows_standalone_bit_exact(kind, count, hops, d, with_batch):
    """ops.hop forward and backward at odd widths, with and without molecule ids (tile windows)."""
    from aimx import ops
    n, edges, batch = _graph(kind, count, hops, seed=d)
    rng = np.random.default_rng(d)
    x = rng.standard_normal((n, d)).astype(np.float32)
    plan = _plan(n, hops, edges, batch if with_batch else None)
    xg = torch.from_numpy(x).to(DEV).requires_grad_()
    out = ops.hop(plan, xg)
    assert np.array_equal(out.detach().cpu().numpy(), _fwd_ref(x, edges[:, 0], edges[:, 1], hops))
    g = rng.standard_normal((hops * n, d)).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    assert np.array_equal(xg.grad.cpu().numpy(), _bwd_ref(g, edges[:, 0], edges[:, 1], n))


def _abi():
    from aimx import _lib
    return _lib.load(), _lib.ptr, _lib.stream_ptr


@pytest.mark.parametrize("d,hops", [(153, 3), (307, 6), (38, 3), (77, 4)])
def test_hop_rows_stack_layouts_bit_exact(d, hops):
    """The stack's calls (stack.hip): the forward writes the hop chunks into F = [x | c_0 | ...]
    (ld D(h+1), chunk j at column (j+1)D: unaligned for odd D); the backward reads F's hop-chunk
    gradients (chunked source rows), adds the chunk-0 gradient and the outer residual and writes
    the layer-below's dY slot (ld 2D, column offset D)."""
    lib, P, S = _abi()
    n, edges, batch = _graph("synth40", 40, hops, seed=d + hops)
    plan = _plan(n, hops, edges, batch)
    seg, seg_st = plan.row_seg()
    K = d * (hops + 1)
    rng = np.random.default_rng(7)
    F = torch.from_numpy(rng.standard_normal((n, K)).astype(np.float32)).to(DEV)
    x = F[:, :d].cpu().numpy()
    keep = F[:, :d].clone()
    rc = lib.aimx_segment_gather_sum(P(F), K, 0, 0, d, P(plan.fwd.rowptr), P(plan.fwd.col), hops * n, P(F) + 4 * d, K,
                                     n, d, None, 0, None, 0, seg, seg_st, S(F.device))
    assert rc == 0
    ref = _fwd_ref(x, edges[:, 0], edges[:, 1], hops)
    Fh = F.cpu().numpy()
    assert torch.equal(F[:, :d], keep)  # chunk 0 untouched
    for j in range(hops):
        assert np.array_equal(Fh[:, (j + 1) * d:(j + 2) * d], ref[j * n:(j + 1) * n]), j
    # backward: dst[j] = (dF[j, :D] + sum_{e: src%N == j} dF_hop[target_e]) + dY[j]
    dF = torch.from_numpy(rng.standard_normal((n, K)).astype(np.float32)).to(DEV)
    dUGy = torch.from_numpy(rng.standard_normal((n, 2 * d)).astype(np.float32)).to(DEV)  # dY = [:, D:]
    dst = torch.full((n, 2 * d), 7.0, device=DEV)
    rc = lib.aimx_segment_gather_sum(P(dF) + 4 * d, K, n, d, d, P(plan.bwd.rowptr), P(plan.bwd.col), n, P(dst) + 4 * d,
                                     2 * d, 0, 0, P(dF), K, P(dUGy) + 4 * d, 2 * d, seg, seg_st, S(F.device))
    assert rc == 0
    dFh = dF.cpu().numpy()
    g = np.concatenate([dFh[:, (j + 1) * d:(j + 2) * d] for j in range(hops)], 0)
    acc = _bwd_ref(g, edges[:, 0], edges[:, 1], n)
    exp = (dFh[:, :d] + acc) + dUGy.cpu().numpy()[:, d:]
    got = dst.cpu().numpy()
    assert np.array_equal(got[:, d:], exp)
    assert np.all(got[:, :d] == 7.0)  # the columns left of the slot untouched


def test_hop_rows_misaligned_bases_bit_exact():
    """Source and output bases at every float offset inside 16 bytes, odd leading dimensions."""
    lib, P, S = _abi()
    n, edges, batch = _graph("synth40", 24, 3, seed=5)
    plan = _plan(n, 3, edges, batch)
    seg, seg_st = plan.row_seg()
    d = 153
    rng = np.random.default_rng(11)
    for off_s in range(4):
        for off_o in range(4):
            ld_s, ld_o = d + 2, d + 1
            xs = torch.from_numpy(rng.standard_normal(n * ld_s + 8).astype(np.float32)).to(DEV)
            out = torch.full((3 * n * ld_o + 8,), 3.0, device=DEV)
            rc = lib.aimx_segment_gather_sum(P(xs) + 4 * off_s, ld_s, 0, 0, d, P(plan.fwd.rowptr), P(plan.fwd.col),
                                             3 * n, P(out) + 4 * off_o, ld_o, n, n * ld_o, None, 0, None, 0, seg, seg_st,
                                             S(xs.device))
            assert rc == 0
            xh = xs.cpu().numpy()[off_s:off_s + n * ld_s].reshape(n, ld_s)[:, :d]
            ref = _fwd_ref(np.ascontiguousarray(xh), edges[:, 0], edges[:, 1], 3)
            oh = out.cpu().numpy()
            body = oh[off_o:off_o + 3 * n * ld_o].reshape(3 * n, ld_o)
            assert np.array_equal(body[:, :d], ref), (off_s, off_o)
            assert np.all(body[:, d:] == 3.0) and np.all(oh[:off_o] == 3.0)  # gaps untouched


@pytest.mark.parametrize("hub_degree", [9, 300, 20_000])
def test_hop_rows_hubs_and_general_bit_exact(hub_degree):
    """Random targets over all hop chunks (non-empty big tiles), src >= N and negative, hub rows
    whose col slice exceeds the LDS capacity (global fallback) — forward and backward, D = 153."""
    from aimx import ops
    rng = np.random.default_rng(hub_degree)
    n, h, d = 3000, 3, 153
    t = np.concatenate([rng.integers(0, h * n, 20_000), np.repeat(rng.choice(n, 5, replace=False), hub_degree)])
    s = rng.integers(-n, 2 * n, t.shape[0])
    perm = rng.permutation(t.shape[0])
    t, s = t[perm], s[perm]
    from aimx.plan import GraphPlan
    plan = GraphPlan(n, h, target=torch.from_numpy(t).to(DEV), src=torch.from_numpy(s).to(DEV))
    x = rng.standard_normal((n, d)).astype(np.float32)
    xg = torch.from_numpy(x).to(DEV).requires_grad_()
    out = ops.hop(plan, xg)
    assert np.array_equal(out.detach().cpu().numpy(), _fwd_ref(x, t, s, h))
    g = rng.standard_normal((h * n, d)).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    assert np.array_equal(xg.grad.cpu().numpy(), _bwd_ref(g, t, s, n))


def test_hop_rows_long_molecule_bit_exact():
    """A 260-atom molecule (longer than a piece and than one 128-row scan window) among 40-atom
    ones: pieces of a molecule, the continued scan, sources wider than the staging capacity."""
    from aimx import ops
    n, edges, batch = _graph("synth40", 40, 3, seed=3)
    batch = batch.copy()
    lo, hi = np.searchsorted(batch, 10), np.searchsorted(batch, 17)
    batch[lo:hi] = 10  # merge molecules 10..16 into one id (edges stay inside it)
    # and one real long molecule: connect the merged atoms in a chain through extra pairs
    extra = np.stack([np.arange(lo + 1, hi), np.arange(lo, hi - 1)], 1)
    edges = np.concatenate([edges, extra, extra[:, ::-1]], 0)
    _, inv = np.unique(batch, return_inverse=True)
    batch = inv.astype(np.int64)
    assert hi - lo > 260
    d = 153
    rng = np.random.default_rng(1)
    x = rng.standard_normal((n, d)).astype(np.float32)
    outs = []
    for b in (batch, None):
        plan = _plan(n, 3, edges, b)
        xg = torch.from_numpy(x).to(DEV).requires_grad_()
        out = ops.hop(plan, xg)
        g = torch.from_numpy(np.random.default_rng(2).standard_normal((3 * n, d)).astype(np.float32)).to(DEV)
        out.backward(g)
        outs.append((out.detach().cpu().numpy(), xg.grad.cpu().numpy()))
    assert np.array_equal(outs[0][0], _fwd_ref(x, edges[:, 0], edges[:, 1], 3))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][1], _bwd_ref(g.cpu().numpy(), edges[:, 0], edges[:, 1], n))


@pytest.mark.parametrize("d,hops,cap", [(76, 3, 37), (153, 3, 101), (307, 6, 64)])
def test_hop_row_range_split_bit_exact(d, hops, cap):
    """A hop launch past the kernels' 32-bit row / thread indexing runs as consecutive row ranges
    inside each output chunk (hop.hip; forced here at `cap` rows per launch through the
    AIMX_HOP_MAX_ROWS option): forward into the stack's chunked F layout and the backward with its
    residual terms are bit-identical to one launch."""
    from aimx import _lib
    lib, P, S = _abi()
    n, edges, batch = _graph("synth40", 30, hops, seed=d)
    plan = _plan(n, hops, edges, batch)
    seg, seg_st = plan.row_seg()
    K = d * (hops + 1)
    rng = np.random.default_rng(3)
    F0 = torch.from_numpy(rng.standard_normal((n, K)).astype(np.float32)).to(DEV)
    dF = torch.from_numpy(rng.standard_normal((n, K)).astype(np.float32)).to(DEV)
    dY = torch.from_numpy(rng.standard_normal((n, 2 * d)).astype(np.float32)).to(DEV)
    res = []
    for opts in ({}, {"AIMX_HOP_MAX_ROWS": cap}):
        with _lib.options(**opts):
            F = F0.clone()
            assert lib.aimx_segment_gather_sum(P(F), K, 0, 0, d, P(plan.fwd.rowptr), P(plan.fwd.col), hops * n,
                                               P(F) + 4 * d, K, n, d, None, 0, None, 0, seg, seg_st, S(DEV)) == 0
            dst = torch.zeros((n, 2 * d), device=DEV)
            assert lib.aimx_segment_gather_sum(P(dF) + 4 * d, K, n, d, d, P(plan.bwd.rowptr), P(plan.bwd.col), n,
                                               P(dst) + 4 * d, 2 * d, 0, 0, P(dF), K, P(dY) + 4 * d, 2 * d, seg,
                                               seg_st, S(DEV)) == 0
            torch.cuda.synchronize()
            res.append((F, dst))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
