"""Autograd operators over the C ABI (include/aimx.h). HIP device only — no CPU fallback.

Each operator corresponds to a reference interface:
  message_passing_stack  <- GNN._message_passing_forward + ShellConvolutionLayer.forward
                            (src/models/gnn.py:276-308, 622-658; src/models/layers.py:63-108)
  hop                    <- ShellConvolutionLayer.message_passing (layers.py:133-167)
  attention_pool         <- MultiHeadAttentionPoolingLayer.forward (pooling.py:122-172)
  segment_pool           <- Mean/Max/SumPoolingLayer.forward (pooling.py:15-80)
  partial_charges        <- GNN._partial_charge_calculation (gnn.py:622-658)
  l1_loss                <- nn.L1Loss / WeightedL1Loss (trainer.py:24-35, models/losses.py:14-48)
"""
from __future__ import annotations

import os

import torch

from . import _lib
from ._lib import ShellStack, ShellStackGrad, check, ptr, ptr_array, stream_ptr

_F32 = torch.float32


class Arena:
    """One allocation carved into 256-byte aligned views (fewer allocator round trips per step)."""

    def __init__(self, device, dtype=_F32):
        self.device, self.dtype = device, dtype
        self.specs = []
        self.total = 0

    def add(self, *shape):
        n = 1
        for s in shape:
            n *= int(s)
        off = self.total
        self.total += (n + 63) // 64 * 64
        self.specs.append((off, n, shape))
        return len(self.specs) - 1

    def alloc(self):
        buf = torch.empty(max(self.total, 64), dtype=self.dtype, device=self.device)
        return buf, [buf.narrow(0, off, n).view(*shape) for off, n, shape in self.specs]


def _rows(t):
    """(tensor, leading dim) for a row-major-compatible 2-D view (stride(1) == 1)."""
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return t, t.stride(0)
    t = t.contiguous()
    return t, t.shape[1]


# ---------------------------------------------------------------------------------------------
# Message-passing stack
# ---------------------------------------------------------------------------------------------
class _MPStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, plan, x_in, total_charges, drop_seed, *params):
        lib = _lib.load()
        dev = x_in.device
        n, d, h, nl, nm = spec["N"], spec["D"], spec["num_hops"], spec["num_layers"], spec["num_mlp"]
        k = d * (h + 1)
        lf, lug, la = _stack_strides(d, k)
        x_in, x_ld = _rows(x_in)
        ar = Arena(dev)
        iF = [ar.add(n, lf) for _ in range(nl)]
        iX = [ar.add(n, d) if (spec["use_pc"] and l > 0) else None for l in range(nl)]
        iUG = [ar.add(n, lug) for _ in range(nl)]
        iU = [ar.add(n, d) for _ in range(nl)]
        iV = [ar.add(n, d) for _ in range(nl * nm)]
        iR = [ar.add(n, la) for _ in range(nl * nm)]
        iA = [ar.add(n, la) if (j % nm) != nm - 1 else None for j in range(nl * nm)]
        buf, views = ar.alloc()
        F = [views[i] for i in iF]
        X = [views[i] if i is not None else None for i in iX]
        UG = [views[i] for i in iUG]
        U = [views[i] for i in iU]
        V = [views[i] for i in iV]
        R = [views[i] for i in iR]
        A = [views[i] if i is not None else None for i in iA]
        # tensors handed to autograd are standalone allocations, never views of the arena
        out = torch.empty(n, d, dtype=_F32, device=dev)
        drop = bool(spec["training"]) and spec["drop_p"] > 0
        M = [torch.empty(n, d, dtype=torch.uint8, device=dev) for _ in range(nl * nm)] if drop else []
        # [input_proj.W ; global_skip_proj.W] and their biases of every layer, packed by ONE cat
        # kernel (layer blocks padded to 64 floats: 16-byte aligned GEMM operands)
        packed, w_ig, b_ig = _pack_ig(params, nl, nm, d, k)
        w1, b1, w2, b2 = [], [], [], []
        for l in range(nl):
            base = l * (4 + 4 * nm) + 4
            for j in range(nm):
                w1.append(params[base + 4 * j])
                b1.append(params[base + 4 * j + 1])
                w2.append(params[base + 4 * j + 2])
                b2.append(params[base + 4 * j + 3])
        s = ShellStack()
        s.N, s.D, s.num_hops, s.num_layers, s.num_mlp = n, d, h, nl, nm
        s.act, s.use_pc, s.training, s.mode_single = spec["act"], int(spec["use_pc"]), int(drop), int(spec["single"])
        s.precision = spec["prec"]
        s.ld_f, s.ld_ug, s.ld_act = lf, lug, la
        s.drop_p = float(spec["drop_p"]) if drop else 0.0
        s.drop_seed = ptr(drop_seed) if drop else None
        s.fwd_rowptr, s.fwd_col = ptr(plan.fwd.rowptr), ptr(plan.fwd.col)
        s.bwd_rowptr, s.bwd_col = ptr(plan.bwd.rowptr), ptr(plan.bwd.col)
        if plan.graph is not None:
            s.gptr, s.gperm, s.G = ptr(plan.graph.rowptr), ptr(plan.graph.col), plan.G
        s.total_charges = ptr(total_charges)
        s.row_seg, s.row_seg_stride = plan.row_seg()
        keep = [ptr_array(w_ig), ptr_array(b_ig), ptr_array(w1), ptr_array(b1), ptr_array(w2), ptr_array(b2),
                ptr_array(F), ptr_array(X), ptr_array(UG), ptr_array(U), ptr_array(V), ptr_array(R), ptr_array(A),
                ptr_array(M)]
        (s.w_ig, s.b_ig, s.w1, s.b1, s.w2, s.b2, s.F, s.X, s.UG, s.U, s.V, s.R, s.A, s.M) = [
            _ct_addr(a) for a in keep]
        s.x_in, s.x_in_ld = ptr(x_in), x_ld
        s.out, s.out_ld = ptr(out), d
        wsb = lib.aimx_shell_stack_workspace_bytes(s)
        ws = torch.empty(max(wsb // 4, 1), dtype=_F32, device=dev)
        s.workspace, s.workspace_bytes = ptr(ws), wsb
        s.counters, s.n_counters = ptr(_lib.counters(dev)), _lib.N_COUNTERS
        check(lib.aimx_shell_stack_forward(s, stream_ptr(dev)), "shell_stack_forward")
        ctx.spec, ctx.plan = spec, plan
        # inputs go through save_for_backward; only forward-internal buffers live on ctx
        ctx.save_for_backward(x_in, total_charges, drop_seed, *params)
        ctx.state = dict(buf=buf, M=M, F=F, X=X, UG=UG, U=U, V=V, R=R, A=A, x_ld=x_ld, ws=ws, drop=drop,
                         packed=packed, w_ig=w_ig, b_ig=b_ig, lf=lf, lug=lug, la=la)
        return out

    @staticmethod
    def backward(ctx, d_out):
        lib = _lib.load()
        st, spec, plan = dict(ctx.state), ctx.spec, ctx.plan
        x_in, tc, seed, *params = ctx.saved_tensors
        nm_ = spec["num_mlp"]
        st["x_in"], st["tc"], st["seed"] = x_in, tc, seed
        for j, key in enumerate(("w1", "b1", "w2", "b2")):
            st[key] = [params[l * (4 + 4 * nm_) + 4 + 4 * q + j] for l in range(spec["num_layers"]) for q in range(nm_)]
        dev = d_out.device
        n, d, h, nl, nm = spec["N"], spec["D"], spec["num_hops"], spec["num_layers"], spec["num_mlp"]
        k = d * (h + 1)
        d_out, d_ld = _rows(d_out)
        # gradients handed to autograd are standalone allocations; the scratch is one buffer
        new = lambda *shape: torch.empty(*shape, dtype=_F32, device=dev)  # noqa: E731
        dx_t = new(n, d)
        d_packed = torch.empty_like(st["packed"])
        blk = st["packed"].numel() // nl
        dw_ig = [d_packed[l * blk:l * blk + 2 * d * k].view(2 * d, k) for l in range(nl)]
        db_ig = [d_packed[l * blk + 2 * d * k:l * blk + 2 * d * k + 2 * d] for l in range(nl)]
        dw1 = [new(d, d) for _ in range(nl * nm)]
        db1 = [new(d) for _ in range(nl * nm)]
        dw2 = [new(d, d) for _ in range(nl * nm)]
        db2 = [new(d) for _ in range(nl * nm)]
        s = ShellStack()
        s.N, s.D, s.num_hops, s.num_layers, s.num_mlp = n, d, h, nl, nm
        s.act, s.use_pc, s.training, s.mode_single = spec["act"], int(spec["use_pc"]), int(st["drop"]), int(spec["single"])
        s.precision = spec["prec"]
        s.ld_f, s.ld_ug, s.ld_act = st["lf"], st["lug"], st["la"]
        s.drop_p = float(spec["drop_p"]) if st["drop"] else 0.0
        s.drop_seed = ptr(st["seed"]) if st["drop"] else None
        s.fwd_rowptr, s.fwd_col = ptr(plan.fwd.rowptr), ptr(plan.fwd.col)
        s.bwd_rowptr, s.bwd_col = ptr(plan.bwd.rowptr), ptr(plan.bwd.col)
        if plan.graph is not None:
            s.gptr, s.gperm, s.G = ptr(plan.graph.rowptr), ptr(plan.graph.col), plan.G
        s.total_charges = ptr(st["tc"])
        s.row_seg, s.row_seg_stride = plan.row_seg()
        keep = [ptr_array(st[nm_]) for nm_ in ("w_ig", "b_ig", "w1", "b1", "w2", "b2", "F", "X", "UG", "U", "V", "R",
                                               "A", "M")]
        (s.w_ig, s.b_ig, s.w1, s.b1, s.w2, s.b2, s.F, s.X, s.UG, s.U, s.V, s.R, s.A, s.M) = [
            _ct_addr(a) for a in keep]
        s.x_in, s.x_in_ld = ptr(st["x_in"]), st["x_ld"]
        s.workspace, s.workspace_bytes = ptr(st["ws"]), st["ws"].numel() * 4
        s.counters, s.n_counters = ptr(_lib.counters(dev)), _lib.N_COUNTERS
        g = ShellStackGrad()
        g.d_out, g.d_out_ld = ptr(d_out), d_ld
        g.d_x_in, g.d_x_in_ld = ptr(dx_t), d
        gkeep = [ptr_array(x) for x in (dw_ig, db_ig, dw1, db1, dw2, db2)]
        g.d_w_ig, g.d_b_ig, g.d_w1, g.d_b1, g.d_w2, g.d_b2 = [_ct_addr(a) for a in gkeep]
        gwsb = lib.aimx_shell_stack_backward_workspace_bytes(s)
        buf = torch.empty(max(gwsb // 4, 1), dtype=_F32, device=dev)
        g.workspace, g.workspace_bytes = ptr(buf), buf.numel() * 4
        check(lib.aimx_shell_stack_backward(s, g, stream_ptr(dev)), "shell_stack_backward")
        grads = []
        for l in range(nl):
            # input_proj / global_skip_proj weight and bias gradients: views of the packed gradient
            grads += [dw_ig[l][:d], dw_ig[l][d:], db_ig[l][:d], db_ig[l][d:]]
            for j in range(nm):
                idx = l * nm + j
                grads += [dw1[idx], db1[idx], dw2[idx], db2[idx]]
        del keep, gkeep, buf
        return (None, None, dx_t, None, None, *grads)


_PAD = {}


def _stack_strides(d, k):
    """Row strides of the stack's F [N, K], UG [N, 2D] and MLP activation (R, A) buffers: rounded up
    to 4 floats, so every row is 16-byte aligned and the weight gradients over them take 16-byte loads
    at odd D (c4 / c5: D = 153 / 307; profiles/r05_wgrad_rows_ab.txt)."""
    r4 = lambda v: -(-v // 4) * 4  # noqa: E731
    return r4(k), r4(2 * d), r4(d)


def _ig_in_place(heads, d, k, blk):
    """The packed [Wi ; Wg ; bi ; bg | pad] x layers block as a view when the parameters already
    sit at exactly those offsets of one storage (GNN.pack_ig_params), else None."""
    t0 = heads[0][0]
    if t0.dtype != _F32 or not t0.is_cuda:
        return None
    st = t0.untyped_storage().data_ptr()
    base = t0.data_ptr()
    offs = (0, d * k, 2 * d * k, 2 * d * k + d)
    for l, ps in enumerate(heads):
        for o, p in zip(offs, ps):
            if p.dtype != _F32 or not p.is_contiguous() or p.untyped_storage().data_ptr() != st or \
                    p.data_ptr() != base + 4 * (l * blk + o):
                return None
    n = len(heads) * blk
    if t0.storage_offset() + n > t0.untyped_storage().nbytes() // 4:
        return None
    return t0.detach().as_strided((n,), (1,))


def pack_ig_params(params, nl, nm, d, k):
    """Lay every layer's [Wi ; Wg ; bi ; bg] out as _pack_ig's packed block (one storage, padded
    64-float layer blocks) and point the Parameters at it (same values, same state_dict), so
    message_passing_stack reads the weights in place instead of a per-step cat."""
    with torch.no_grad():
        packed, _, _ = _pack_ig(params, nl, nm, d, k)
        per = 2 * d * k + 2 * d
        blk = (per + 63) // 64 * 64
        packed = packed.clone()
        offs = (0, d * k, 2 * d * k, 2 * d * k + d)
        for l in range(nl):
            for o, p in zip(offs, params[l * (4 + 4 * nm):l * (4 + 4 * nm) + 4]):
                p.data = packed[l * blk + o:l * blk + o + p.numel()].view(p.shape)


def _pack_ig(params, nl, nm, d, k):
    """One cat of every layer's [Wi ; Wg] (each [D, K]) and [bi ; bg]: returns (packed, w_ig views
    [2D, K], b_ig views [2D]); per-layer blocks are padded to a multiple of 64 floats."""
    per = 2 * d * k + 2 * d
    blk = (per + 63) // 64 * 64
    dev = params[0].device
    parts = []
    pad = None
    if blk > per:
        pad = _PAD.get((dev, blk - per))
        if pad is None:
            pad = torch.zeros(blk - per, dtype=_F32, device=dev)
            _PAD[(dev, blk - per)] = pad
    heads = [params[l * (4 + 4 * nm):l * (4 + 4 * nm) + 4] for l in range(nl)]
    packed = _ig_in_place(heads, d, k, blk)
    if packed is not None:  # GNN.pack_ig_params laid the parameters out this way: no cat
        w_ig = [packed[l * blk:l * blk + 2 * d * k].view(2 * d, k) for l in range(nl)]
        b_ig = [packed[l * blk + 2 * d * k:l * blk + per] for l in range(nl)]
        return packed, w_ig, b_ig
    for wi, wg, bi, bg in heads:
        parts += [wi.detach().reshape(-1), wg.detach().reshape(-1), bi.detach().reshape(-1), bg.detach().reshape(-1)]
        if pad is not None:
            parts.append(pad)
    packed = torch.cat(parts)
    w_ig = [packed[l * blk:l * blk + 2 * d * k].view(2 * d, k) for l in range(nl)]
    b_ig = [packed[l * blk + 2 * d * k:l * blk + per] for l in range(nl)]
    return packed, w_ig, b_ig


class _Stereo(torch.autograd.Function):
    """[x | cis/trans | tetrahedral] features (gnn.py:310-326 before stereochemical_embedding_2),
    aimx_stereo_forward / _backward (csrc/stereo.hip)."""

    @staticmethod
    def forward(ctx, x, tet, cis, trans):
        from .plan import build_csr, _zero_status
        import ctypes
        lib = _lib.load()
        x, ldx = _rows(x)
        n, d = x.shape
        dev = x.device
        tet = tet.to(torch.int64).contiguous() if tet.numel() else tet.new_empty(0, 4, dtype=torch.int64)
        m = tet.shape[0] if tet.numel() else 0
        a = _lib.Stereo()
        a.x, a.ldx, a.N, a.D = ptr(x), ldx, n, d
        keep = [x, tet]
        if m:
            status = torch.empty(1, dtype=torch.int32, device=dev)
            csr = build_csr(tet.data_ptr(), 1, 0, None, 0, 0, 4 * m, n, dev, status)
            scratch = torch.empty(4 * m, d, dtype=_F32, device=dev)
            stats = torch.empty(m, 8, dtype=_F32, device=dev)
            a.tet, a.tet_stride0, a.tet_stride1, a.M = ptr(tet), 4, 1, m
            a.t_rowptr, a.t_col, a.scratch, a.stats = ptr(csr.rowptr), ptr(csr.col), ptr(scratch), ptr(stats)
            keep += [csr.rowptr, csr.col, stats]
        for name, t in (("cis", cis), ("trans", trans)):
            if t.numel():
                if t.dim() != 2 or t.shape[0] < 2 or t.dtype != torch.int64:
                    raise _lib.AimxError(f"aimx.stereo: {name} must be int64 [rows >= 2, cols] (the reference "
                                         f"reads rows 0 and 1)")
                setattr(a, name, ptr(t))
                setattr(a, name + "_stride0", t.stride(0))
                setattr(a, name + "_stride1", t.stride(1))
                setattr(a, "n_" + name, t.shape[0])
                keep.append(t)
        out = torch.empty(n, 3 * d, dtype=_F32, device=dev)
        a.out, a.ldo = ptr(out), 3 * d
        check(lib.aimx_stereo_forward(ctypes.byref(a), stream_ptr(dev)), "stereo_forward")
        ctx.args, ctx.keep, ctx.m, ctx.shape = a, keep, m, (n, d)
        return out

    @staticmethod
    def backward(ctx, g):
        import ctypes
        lib = _lib.load()
        n, d = ctx.shape
        g = g.contiguous()
        dx = torch.empty(n, d, dtype=_F32, device=g.device)
        gs = torch.empty(max(4 * ctx.m, 1), d, dtype=_F32, device=g.device)
        check(lib.aimx_stereo_backward(ctypes.byref(ctx.args), ptr(g), 3 * d, ptr(dx), d, ptr(gs),
                                       stream_ptr(g.device)), "stereo_backward")
        return dx, None, None, None


def stereo_features(x, tet, cis, trans):
    """[x | cis_trans(x) | tetrahedral(x)] ([N, 3D]) of the reference's stereochemistry
    (gnn.py:310-497) on the HIP kernels; differentiable in x."""
    _lib.require_device(x)
    if x.dtype != _F32:
        raise _lib.AimxError("aimx.stereo: fp32 features")
    return _Stereo.apply(x, tet, cis, trans)


def _seed_state(owner, device):
    st = getattr(owner, "_aimx_seed_state", None)
    if st is None or st.device != device:
        st = torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)
        owner._aimx_seed_state = st
    return st


def dropout_seeds(owner, n, device):
    """n int64 dropout seeds for one forward, drawn on the device from a counter kept on `owner`
    (aimx_dropout_seeds; one launch, graph-safe). The counter starts from torch's generator."""
    st = _seed_state(owner, device)
    seeds = torch.empty(n, dtype=torch.int64, device=device)
    check(_lib.load().aimx_dropout_seeds(ptr(st), ptr(seeds), int(n), stream_ptr(device)), "dropout_seeds")
    return seeds


def dropout_seed_slots(owner, n, device):
    """(counter, seeds) for embed_project(..., seeds=...): the same draw as dropout_seeds, done by
    the embedding gather's launch instead of a launch of its own."""
    return _seed_state(owner, device), torch.empty(n, dtype=torch.int64, device=device)


def _ct_addr(arr):
    import ctypes
    return ctypes.cast(arr, ctypes.c_void_p).value


def message_passing_stack(plan, x, params, *, num_hops, num_layers, num_mlp, act, use_pc=False, total_charges=None,
                          training=False, drop_p=0.0, drop_seed=None, single=False):
    """params: per layer [input_proj.W (D,K), global_skip_proj.W (D,K), input_proj.b, global_skip_proj.b,
    then per MLP block w1, b1, w2, b2] (ShellConvolutionLayer._aimx_params())."""
    _lib.require_device(x)
    if x.dtype != _F32:
        raise _lib.AimxError("aimx: message passing runs in fp32 (the reference dtype)")
    n, d = x.shape
    spec = dict(N=n, D=d, num_hops=num_hops, num_layers=num_layers, num_mlp=num_mlp, act=_lib.ACT_KIND[act]
                if isinstance(act, str) else int(act), use_pc=bool(use_pc), training=bool(training),
                drop_p=float(drop_p), single=bool(single), prec=amp_precision())
    if use_pc and (plan.graph is None or total_charges is None):
        raise _lib.AimxError("aimx: partial charges need batch indices and total charges")
    tc = total_charges.contiguous().float() if total_charges is not None else None
    return _MPStack.apply(spec, plan, x, tc, drop_seed, *params)


# ---------------------------------------------------------------------------------------------
# The hop alone (ShellConvolutionLayer.message_passing)
# ---------------------------------------------------------------------------------------------
class _Hop(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, x):
        lib = _lib.load()
        n, d = x.shape
        h = plan.num_hops
        x, ldx = _rows(x)
        out = torch.empty(h * n, d, dtype=_F32, device=x.device)
        # out viewed as h chunks of n rows (same addresses): tells the kernel where chunk 0 ends
        seg, seg_st = plan.row_seg()
        check(lib.aimx_segment_gather_sum(ptr(x), ldx, 0, 0, d, ptr(plan.fwd.rowptr), ptr(plan.fwd.col), h * n,
                                          ptr(out), d, n, n * d, None, 0, None, 0, seg, seg_st,
                                          stream_ptr(x.device)), "hop_forward")
        ctx.plan = plan
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        plan = ctx.plan
        n = plan.N
        g = g.contiguous()
        d = g.shape[1]
        dx = torch.empty(n, d, dtype=_F32, device=g.device)
        seg, seg_st = plan.row_seg()
        check(lib.aimx_segment_gather_sum(ptr(g), d, 0, 0, d, ptr(plan.bwd.rowptr), ptr(plan.bwd.col), n, ptr(dx), d,
                                          0, 0, None, 0, None, 0, seg, seg_st, stream_ptr(g.device)), "hop_backward")
        return None, dx


def hop(plan, x):
    """[num_hops*N, D] = scatter_add(x[src % N], target) (bit-exact in edge order)."""
    _lib.require_device(x)
    return _Hop.apply(plan, x)


# ---------------------------------------------------------------------------------------------
# Attention pooling
# ---------------------------------------------------------------------------------------------
class _AttnPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, x, W, b, tau):
        lib = _lib.load()
        x, ldx = _rows(x)
        n, c = x.shape
        H = W.shape[0]
        G = plan.G
        W = W.contiguous()
        b = b.contiguous()
        tau = tau.contiguous().float()
        pooled = torch.empty(G, c, dtype=_F32, device=x.device)
        attn = torch.empty(H, n, dtype=_F32, device=x.device)
        scores = torch.empty(H, n, dtype=_F32, device=x.device)
        check(lib.aimx_attn_pool_forward(ptr(x), ldx, n, c, ptr(W), ptr(b), ptr(tau), H, ptr(plan.graph.rowptr),
                                         ptr(plan.graph.col), G, ptr(pooled), ptr(attn), ptr(scores),
                                         stream_ptr(x.device)), "attn_pool_forward")
        ctx.plan = plan
        ctx.ldx = ldx
        ctx.save_for_backward(x, W, tau, attn, scores)
        ctx.set_materialize_grads(False)  # an unused attention output needs no zero-filled gradient
        return pooled, attn

    @staticmethod
    def backward(ctx, d_pooled, d_attn):
        lib = _lib.load()
        x, W, tau, attn, scores = ctx.saved_tensors
        plan = ctx.plan
        n, c = x.shape
        H = W.shape[0]
        G = plan.G
        dev = x.device
        if d_pooled is None:
            d_pooled = torch.zeros(G, c, dtype=_F32, device=dev)
        d_pooled = d_pooled.contiguous()
        d_attn = d_attn.contiguous() if d_attn is not None else None
        dx = torch.empty(n, c, dtype=_F32, device=dev)  # every atom row is written (its molecule's segment)
        dW = torch.empty(H, c, dtype=_F32, device=dev)
        db = torch.empty(H, dtype=_F32, device=dev)
        dtau = torch.empty(1, dtype=_F32, device=dev)
        wsb = lib.aimx_attn_pool_workspace_bytes(n, c, H, G)
        ws = torch.empty(wsb // 4 + 1, dtype=_F32, device=dev)
        check(lib.aimx_attn_pool_backward(ptr(x), ctx.ldx, n, c, ptr(W), ptr(tau), H, ptr(plan.graph.rowptr),
                                          ptr(plan.graph.col), G, ptr(attn), ptr(scores), ptr(d_pooled), ptr(d_attn),
                                          ptr(dx), c, ptr(dW), ptr(db), ptr(dtau), ptr(ws), wsb, stream_ptr(dev)),
              "attn_pool_backward")
        return None, dx, dW, db, dtau.view(())


def attention_pool(plan, x, W, b, tau):
    _lib.require_device(x, W, b, tau)
    return _AttnPool.apply(plan, x, W, b, tau)


def _packed_rows(ts):
    """The [len(ts), k] tensor the row tensors ts (each k elements) already form in memory (one
    contiguous storage, consecutive, in order), or None."""
    t0 = ts[0]
    k = t0.numel()
    base = t0.data_ptr()
    for i, t in enumerate(ts):
        if t.numel() != k or not t.is_contiguous() or t.data_ptr() != base + i * k * t.element_size() or \
                t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr() or t.dtype != t0.dtype:
            return None
    return t0.detach().as_strided((len(ts), k), (k, 1))


class _AttnPoolHeads(torch.autograd.Function):
    """Attention pool over per-head Linear(C, 1) parameters (pooling.py:122-172's ModuleList) laid out
    as one [H, C] / [H] block (MultiHeadAttentionPoolingLayer packs them): the kernels read that
    block in place and the gradients come back as row views of one [H, C] / [H] result, so neither
    direction launches a cat or a split."""

    @staticmethod
    def forward(ctx, plan, x, W, b, tau, *heads):
        pooled, attn = _AttnPool.forward(ctx, plan, x, W, b, tau)
        ctx.H = len(heads) // 2
        return pooled, attn

    @staticmethod
    def backward(ctx, d_pooled, d_attn):
        _, dx, dW, db, dtau = _AttnPool.backward(ctx, d_pooled, d_attn)
        H = ctx.H
        return (None, dx, None, None, dtau) + tuple(dW[i:i + 1] for i in range(H)) + \
            tuple(db[i:i + 1] for i in range(H))


def attention_pool_heads(plan, x, weights, biases, tau):
    """attention_pool with the H head weights [1, C] and biases [1] given separately (the
    reference's nn.Linear per head); no concatenation when they are packed (_packed_rows)."""
    W, b = _packed_rows(weights), _packed_rows(biases)
    if W is None or b is None:
        return attention_pool(plan, x, torch.cat(list(weights), 0), torch.cat(list(biases), 0), tau)
    _lib.require_device(x, W, b, tau)
    return _AttnPoolHeads.apply(plan, x, W, b.view(-1), tau, *weights, *biases)


# ---------------------------------------------------------------------------------------------
# Mean / max / sum pooling
# ---------------------------------------------------------------------------------------------
_POOL_KIND = {"mean": 0, "max": 1, "sum": 2}


class _SegPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, kind, x):
        lib = _lib.load()
        x, ldx = _rows(x)
        n, c = x.shape
        G = plan.G
        out = torch.empty(G, c, dtype=_F32, device=x.device)
        am = torch.empty(G, c, dtype=torch.int32, device=x.device) if kind == 1 else None
        check(lib.aimx_segment_pool_forward(kind, ptr(x), ldx, n, c, ptr(plan.graph.rowptr), ptr(plan.graph.col), G,
                                            ptr(out), ptr(am), stream_ptr(x.device)), "segment_pool_forward")
        ctx.plan, ctx.kind, ctx.n = plan, kind, n
        ctx.am = am
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        plan = ctx.plan
        g = g.contiguous()
        c = g.shape[1]
        dx = torch.zeros(ctx.n, c, dtype=_F32, device=g.device)
        check(lib.aimx_segment_pool_backward(ctx.kind, ptr(g), ctx.n, c, ptr(plan.graph.rowptr), ptr(plan.graph.col),
                                             plan.G, ptr(ctx.am), ptr(dx), c, stream_ptr(g.device)),
              "segment_pool_backward")
        return None, None, dx


def segment_pool(plan, kind, x):
    _lib.require_device(x)
    return _SegPool.apply(plan, _POOL_KIND[kind], x)


# ---------------------------------------------------------------------------------------------
# Partial charges (standalone; fused inside the stack otherwise)
# ---------------------------------------------------------------------------------------------
class _Charges(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, x, total_charges):
        lib = _lib.load()
        x, ldx = _rows(x)
        n, d = x.shape
        tc = total_charges.contiguous().float()
        out = torch.empty(n, d, dtype=_F32, device=x.device)
        check(lib.aimx_partial_charge_forward(ptr(x), ldx, n, d, ptr(plan.graph.rowptr), ptr(plan.graph.col), plan.G,
                                              ptr(tc), ptr(out), d, stream_ptr(x.device)), "partial_charge_forward")
        ctx.plan, ctx.ldx = plan, ldx
        ctx.save_for_backward(x, tc)
        return out

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        x, tc = ctx.saved_tensors
        plan = ctx.plan
        g = g.contiguous()
        n, d = g.shape
        dx = torch.zeros(n, d, dtype=_F32, device=g.device)
        check(lib.aimx_partial_charge_backward(ptr(x), ctx.ldx, n, d, ptr(plan.graph.rowptr), ptr(plan.graph.col),
                                               plan.G, ptr(tc), ptr(g), d, ptr(dx), d, stream_ptr(g.device)),
              "partial_charge_backward")
        return None, dx, None


def partial_charges(plan, x, total_charges):
    _lib.require_device(x, total_charges)
    return _Charges.apply(plan, x, total_charges)


# ---------------------------------------------------------------------------------------------
# Dense layers on the fused fp32 MFMA GEMM (nn.Linear semantics, optional fused activation)
# ---------------------------------------------------------------------------------------------
PREC_FP32, PREC_BF16 = 0, 1  # AimxGemmArgs.precision (include/aimx.h)


def amp_precision():
    """The GEMM precision of the reference's --mixed_precision path (trainer.py:134): inside
    torch.autocast('cuda') the node-update / dense GEMMs take bf16 operands (fp32 accumulation and
    fp32 outputs; whatever the autocast dtype, bf16 is the MI355X choice: fp32 range, no loss
    scaling needed); otherwise exact fp32, the parity path. Autograd Functions record it at
    forward (ctx.prec) and their backward GEMMs use the same."""
    return PREC_BF16 if torch.is_autocast_enabled("cuda") else PREC_FP32


def _gemm_args(M, N, K, prec=PREC_FP32):
    a = _lib.GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.act, a.dact_kind = -1, -1
    a.precision = prec
    return a


def _run_gemm(a, dev):
    import ctypes
    lib = _lib.load()
    a.counters, a.n_counters = ptr(_lib.counters(dev)), _lib.N_COUNTERS
    wsb = lib.aimx_gemm_workspace_bytes(ctypes.byref(a))
    ws = None
    if wsb:
        ws = torch.empty(wsb // 4 + 1, dtype=_F32, device=dev)
        a.workspace, a.workspace_bytes = ws.data_ptr(), wsb
    check(lib.aimx_gemm(ctypes.byref(a), stream_ptr(dev)), "gemm")
    return ws


def gemm_linear_fwd(x, ldx, W, b, out, ldo, act=-1, pre=None, prec=PREC_FP32):
    """out[M, n_out] = act(x[M, n_in] W^T + b)  (pre-activation to `pre` when act >= 0)."""
    M, n_in = x.shape
    n_out = W.shape[0]
    a = _gemm_args(M, n_out, n_in, prec)
    a.A, a.sam, a.sak = ptr(x), ldx, 1
    a.B, a.sbk, a.sbn = ptr(W), 1, n_in
    a.C, a.ldc = ptr(out), ldo
    a.bias = ptr(b)
    if act >= 0:
        a.act, a.act_ncols = act, n_out
        if pre is not None:
            a.pre, a.ldpre = ptr(pre), n_out
    return _run_gemm(a, x.device)


def gemm_linear_bwd(dy, ldy, x, ldx, W, dx, dW, db, prec=PREC_FP32):
    """dx = dy W ; dW = dy^T x ; db = sum_rows dy (ones-column fusion, split-K)."""
    M, n_out = dy.shape
    n_in = W.shape[1]
    dev = dy.device
    if dx is not None:
        a = _gemm_args(M, n_in, n_out, prec)
        a.A, a.sam, a.sak = ptr(dy), ldy, 1
        a.B, a.sbk, a.sbn = ptr(W), n_in, 1
        a.C, a.ldc = ptr(dx), n_in
        _run_gemm(a, dev)
    a = _gemm_args(n_out, n_in + 1, M, prec)
    a.A, a.sam, a.sak = ptr(dy), 1, ldy
    a.B, a.sbk, a.sbn = ptr(x), ldx, 1
    a.C, a.ldc = ptr(dW), n_in
    a.ones_col, a.col_out = 1, ptr(db)
    _run_gemm(a, dev)


def act_backward(kind, dy, pre):
    lib = _lib.load()
    dy, ldy = _rows(dy)
    out = torch.empty(pre.shape, dtype=_F32, device=pre.device)
    check(lib.aimx_act_backward(kind, ptr(dy), ldy, ptr(pre), pre.shape[1], pre.shape[0], pre.shape[1], ptr(out),
                                pre.shape[1], stream_ptr(pre.device)), "act_backward")
    return out


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, act):
        shape = x.shape
        x2, ldx = _rows(x.reshape(-1, shape[-1]))
        M = x2.shape[0]
        out = torch.empty(M, W.shape[0], dtype=_F32, device=x.device)
        pre = torch.empty_like(out) if act >= 0 else None
        ctx.prec = amp_precision()
        gemm_linear_fwd(x2, ldx, W.contiguous(), b.contiguous() if b is not None else None, out, W.shape[0], act, pre,
                        ctx.prec)
        ctx.act, ctx.ldx, ctx.shape, ctx.has_b = act, ldx, shape, b is not None
        ctx.save_for_backward(x2, W, pre)
        return out.view(*shape[:-1], W.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, W, pre = ctx.saved_tensors
        dy2 = dy.reshape(-1, W.shape[0])
        if ctx.act >= 0:
            dy2 = act_backward(ctx.act, dy2, pre)
        dy2, ldy = _rows(dy2)
        dx = torch.empty(x2.shape[0], W.shape[1], dtype=_F32, device=dy.device) if ctx.needs_input_grad[0] else None
        dW = torch.empty_like(W)
        db = torch.empty(W.shape[0], dtype=_F32, device=dy.device)
        gemm_linear_bwd(dy2, ldy, x2, ctx.ldx, W.contiguous(), dx, dW, db, ctx.prec)
        dx = dx.view(*ctx.shape[:-1], W.shape[1]) if dx is not None else None
        return dx, dW, (db if ctx.has_b else None), None


def linear(x, W, b=None, act=None):
    """y = act(x W^T + b) on the MFMA GEMM (act: None or an activation name)."""
    _lib.require_device(x, W)
    kind = -1 if act is None else (_lib.ACT_KIND[act] if isinstance(act, str) else int(act))
    if b is None:
        raise _lib.AimxError("aimx.linear: bias-free layers are not used on the hot path")
    return _Linear.apply(x, W, b, kind)


# ---------------------------------------------------------------------------------------------
# Atom-feature embeddings + projection (gnn.py:221-225 fused)
# ---------------------------------------------------------------------------------------------
def _tables_struct(indices, tables, grads=None):
    t = _lib.EmbeddingTables()
    t.n_tables = len(tables)
    t.dim = tables[0].shape[1]
    for i, (ix, tb) in enumerate(zip(indices, tables)):
        t.table[i] = ptr(tb)
        t.index[i] = ptr(ix)
        t.rows[i] = tb.shape[0]
        if grads is not None:
            t.grad[i] = ptr(grads[i])
    return t


def _act_backward_into(kind, dy, pre, out):
    """out = dy * act'(pre) for 2-D views with unit column stride (any row strides)."""
    lib = _lib.load()
    dy, ldy = _rows(dy)
    check(lib.aimx_act_backward(kind, ptr(dy), ldy, ptr(pre), pre.stride(0), pre.shape[0], pre.shape[1], ptr(out),
                                out.stride(0), stream_ptr(pre.device)), "act_backward")


class _EmbedProject(torch.autograd.Function):
    @staticmethod
    def forward(ctx, indices, act, split, seeds, W, b, *tables):
        import ctypes
        lib = _lib.load()
        dev = W.device
        idx = [i if i.dtype == torch.int64 else i.long() for i in indices]
        idx = [i.contiguous() for i in idx]
        tables = [t.contiguous() for t in tables]
        n = idx[0].shape[0]
        width = len(tables) * tables[0].shape[1]
        E = torch.empty(n, width, dtype=_F32, device=dev)
        ts = _tables_struct(idx, tables)
        if seeds is not None:  # the forward's dropout seeds ride in the gather launch
            ts.seed_state, ts.seeds, ts.n_seeds = ptr(seeds[0]), ptr(seeds[1]), seeds[1].numel()
        check(lib.aimx_embedding_gather(ctypes.byref(ts), n, ptr(E), width, stream_ptr(dev)), "embedding_gather")
        out = torch.empty(n, W.shape[0], dtype=_F32, device=dev)
        pre = torch.empty_like(out) if act >= 0 else None
        ctx.prec = amp_precision()
        gemm_linear_fwd(E, width, W.contiguous(), b.contiguous(), out, W.shape[0], act, pre, ctx.prec)
        ctx.act = act
        ctx.idx = idx
        ctx.split = split
        ctx.save_for_backward(E, W, pre, *tables)
        if split:  # [x_self | x_other] as two views (gnn.py:227-231): their gradients need no cat
            return out[:, :split], out[:, split:]
        return out

    @staticmethod
    def backward(ctx, *grads):
        import ctypes
        lib = _lib.load()
        E, W, pre, *tables = ctx.saved_tensors
        dev = E.device
        if ctx.split:
            xs = ctx.split
            n, width = E.shape[0], W.shape[0]
            parts = [g if g is not None else torch.zeros(n, w, dtype=_F32, device=dev)
                     for g, w in zip(grads, (xs, width - xs))]
            if ctx.act >= 0 and width % 4:  # act' per part, into the two column ranges of dpre
                dpre = torch.empty(n, width, dtype=_F32, device=dev)
                _act_backward_into(ctx.act, parts[0], pre[:, :xs], dpre[:, :xs])
                _act_backward_into(ctx.act, parts[1], pre[:, xs:], dpre[:, xs:])
            elif ctx.act >= 0:  # act' over both parts into dpre in one launch (the two column sources)
                dpre = torch.empty(n, width, dtype=_F32, device=dev)
                d0, ld0 = _rows(parts[0])
                d1, ld1 = _rows(parts[1])
                check(lib.aimx_act_backward2(ctx.act, ptr(d0), ld0, xs, ptr(d1), ld1, ptr(pre), pre.stride(0), n,
                                             width, ptr(dpre), dpre.stride(0), stream_ptr(dev)), "act_backward2")
            else:
                dpre = torch.cat(parts, dim=1)
        else:
            dy = grads[0]
            dpre = act_backward(ctx.act, dy, pre) if ctx.act >= 0 else dy.contiguous()
        dE = torch.empty_like(E)
        dW = torch.empty_like(W)
        db = torch.empty(W.shape[0], dtype=_F32, device=dev)
        gemm_linear_bwd(dpre, dpre.shape[1], E, E.shape[1], W.contiguous(), dE, dW, db, ctx.prec)
        grads = [torch.empty_like(t) for t in tables]
        ts = _tables_struct(ctx.idx, tables, grads)
        wsb = lib.aimx_embedding_backward_workspace_bytes(ctypes.byref(ts), E.shape[0])
        ws = torch.empty(wsb // 4 + 1, dtype=_F32, device=dev)
        check(lib.aimx_embedding_backward(ctypes.byref(ts), E.shape[0], ptr(dE), dE.shape[1], ptr(ws), wsb,
                                          stream_ptr(dev)), "embedding_backward")
        return (None, None, None, None, dW, db, *grads)


def embed_project(indices, tables, W, b, act=None, split=None, seeds=None):
    """act(cat_t(table_t[indices_t]) W^T + b) — gather, GEMM and activation on the device.
    split=k: returns the column views (out[:, :k], out[:, k:]) (gnn.py:227-231's torch.split) whose
    gradients the backward takes separately (no concatenation launch). seeds=(counter, out) from
    dropout_seed_slots: the gather launch also draws the forward's dropout seeds into out."""
    _lib.require_device(W, *indices)
    kind = -1 if act is None else _lib.ACT_KIND[act]
    return _EmbedProject.apply(list(indices), kind, int(split) if split else 0, seeds, W, b, *tables)


# ---------------------------------------------------------------------------------------------
# Grouped weight gradients (aimx_wgrad_grouped) and the fused LinearBlock (layers.py:170-219)
# ---------------------------------------------------------------------------------------------
def wgrad_grouped(problems):
    """problems: list of (dY [K, M] (ld), X [K, N] (ld), dW [M, N] out, db [M] out or None), all on one
    device; every dW = dY^T X (and db = sum_k dY) in one launch."""
    lib = _lib.load()
    n = len(problems)
    arr = (_lib.WgradProblem * n)()
    dev = problems[0][0].device
    for i, (dy, x, dw, db) in enumerate(problems):
        dy, ldy = _rows(dy)
        x, ldx = _rows(x)
        arr[i].dY, arr[i].ld_dy = ptr(dy), ldy
        arr[i].X, arr[i].ld_x = ptr(x), ldx
        arr[i].dW, arr[i].ld_dw = ptr(dw), dw.shape[1]
        arr[i].col_out = ptr(db)
        arr[i].M, arr[i].N, arr[i].K = dy.shape[1], x.shape[1], dy.shape[0]
    wsb = lib.aimx_wgrad_grouped_workspace_bytes(arr, n)
    ws = torch.empty(max(wsb // 4, 1), dtype=_F32, device=dev)
    check(lib.aimx_wgrad_grouped(arr, n, ptr(ws), ws.numel() * 4, ptr(_lib.counters(dev)), _lib.N_COUNTERS,
                                 stream_ptr(dev)), "wgrad_grouped")
    return ws


class _LinearBlock(torch.autograd.Function):
    """y = linear2(dropout(act(linear1(x)))) [+ x]: two fused GEMMs forward (bias, activation,
    pre-activation store and hash dropout in the first epilogue; bias and skip in the second), two
    input-gradient GEMMs with act'/mask fused, and both weight gradients in one grouped launch."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, act, drop_p, skip, seed):
        ctx.prec = amp_precision()
        dev = x.device
        shape = x.shape
        x2, ldx = _rows(x.reshape(-1, shape[-1]))
        M, n_in = x2.shape
        n_out = W1.shape[0]
        W1, b1, W2, b2 = W1.contiguous(), b1.contiguous(), W2.contiguous(), b2.contiguous()
        H = torch.empty(M, n_out, dtype=_F32, device=dev)
        V = torch.empty(M, n_out, dtype=_F32, device=dev)
        drop = seed is not None and drop_p > 0
        mask = torch.empty(M, n_out, dtype=torch.uint8, device=dev) if drop else None
        a = _gemm_args(M, n_out, n_in, ctx.prec)
        a.A, a.sam, a.sak = ptr(x2), ldx, 1
        a.B, a.sbk, a.sbn = ptr(W1), 1, n_in
        a.C, a.ldc = ptr(H), n_out
        a.bias = ptr(b1)
        a.act, a.act_ncols, a.pre, a.ldpre = act, n_out, ptr(V), n_out
        if drop:
            a.drop_p, a.drop_seed, a.drop_salt = float(drop_p), ptr(seed), 0x5EED
            a.mask_out, a.ldmask = ptr(mask), n_out
        _run_gemm(a, dev)
        Y = torch.empty(M, n_out, dtype=_F32, device=dev)
        a = _gemm_args(M, n_out, n_out, ctx.prec)
        a.A, a.sam, a.sak = ptr(H), n_out, 1
        a.B, a.sbk, a.sbn = ptr(W2), 1, n_out
        a.C, a.ldc = ptr(Y), n_out
        a.bias = ptr(b2)
        if skip:
            a.res[0], a.ldres[0] = ptr(x2), ldx
        _run_gemm(a, dev)
        ctx.act, ctx.drop_p, ctx.skip, ctx.shape = act, float(drop_p), skip, shape
        ctx.save_for_backward(x2, W1, W2, H, V, mask)
        return Y.view(*shape[:-1], n_out)

    @staticmethod
    def backward(ctx, dy):
        x2, W1, W2, H, V, mask = ctx.saved_tensors
        dev = dy.device
        M, n_in = x2.shape
        n_out = W1.shape[0]
        dY, ldy = _rows(dy.reshape(-1, n_out))
        dV = torch.empty(M, n_out, dtype=_F32, device=dev)
        a = _gemm_args(M, n_out, n_out, ctx.prec)  # dV = (dY W2) * mask/(1-p) * act'(V)
        a.A, a.sam, a.sak = ptr(dY), ldy, 1
        a.B, a.sbk, a.sbn = ptr(W2), n_out, 1
        a.C, a.ldc = ptr(dV), n_out
        if mask is not None:
            a.drop_p, a.mask_in, a.ldmask = ctx.drop_p, ptr(mask), n_out
        a.dact_pre, a.lddact, a.dact_kind = ptr(V), n_out, ctx.act
        _run_gemm(a, dev)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, n_in, dtype=_F32, device=dev)
            a = _gemm_args(M, n_in, n_out, ctx.prec)  # dx = dV W1 [+ dY]
            a.A, a.sam, a.sak = ptr(dV), n_out, 1
            a.B, a.sbk, a.sbn = ptr(W1), n_in, 1
            a.C, a.ldc = ptr(dx), n_in
            if ctx.skip:
                a.res[0], a.ldres[0] = ptr(dY), ldy
            _run_gemm(a, dev)
            dx = dx.view(*ctx.shape[:-1], n_in)
        dW1, db1 = torch.empty_like(W1), torch.empty(n_out, dtype=_F32, device=dev)
        dW2, db2 = torch.empty_like(W2), torch.empty(n_out, dtype=_F32, device=dev)
        wgrad_grouped([(dY, H, dW2, db2), (dV, x2, dW1, db1)])
        return dx, dW1, db1, dW2, db2, None, None, None, None


def linear_block(x, W1, b1, W2, b2, act, drop_p=0.0, training=False, skip=False, seed=None):
    """reference LinearBlock.forward (layers.py:204-219) with skip_proj = None. seed: optional
    int64 [1] device tensor for the dropout hash (drawn here when None and dropout is active)."""
    _lib.require_device(x, W1, W2)
    kind = _lib.ACT_KIND[act] if isinstance(act, str) else int(act)
    if not (training and drop_p > 0):
        seed = None
    elif seed is None:
        seed = torch.randint(0, 2 ** 62, (1,), device=x.device, dtype=torch.int64)
    return _LinearBlock.apply(x, W1, b1, W2, b2, kind, float(drop_p), bool(skip), seed)


# ---------------------------------------------------------------------------------------------
# L1 losses (trainer.py:24-35: nn.L1Loss; models/losses.py:14-48: WeightedL1Loss)
# ---------------------------------------------------------------------------------------------
class _L1Loss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, weights, per_sample, rows, accum, grad_of):
        import ctypes
        lib = _lib.load()
        p, ldp = _rows(pred.reshape(pred.shape[0], -1) if pred.dim() != 2 else pred)
        t, ldt = _rows(target.reshape(target.shape[0], -1) if target.dim() != 2 else target)
        total, cols = p.shape
        rows = total if rows is None else rows
        w = weights.contiguous().float() if weights is not None else None
        loss = torch.empty((), dtype=_F32, device=pred.device)
        acc = None
        ctx.pre = None
        if accum is not None:
            loss_sum, nan_count, steps, scale = accum
            acc = _lib.LossAccum(ptr(loss_sum), ptr(nan_count), ptr(steps), float(scale))
            if grad_of is not None:  # the backward's d_pred for that upstream gradient, in this launch
                dp = torch.empty(total, cols, dtype=_F32, device=pred.device)
                acc.d_loss, acc.d_pred, acc.ldd, acc.rows_total = ptr(grad_of), ptr(dp), cols, total
                ctx.pre = (dp, grad_of.data_ptr(), grad_of._version)
        check(lib.aimx_l1_loss_forward_accum(ptr(p), ldp, ptr(t), ldt, rows, cols, ptr(w), int(per_sample), ptr(loss),
                                             ctypes.byref(acc) if acc is not None else None,
                                             stream_ptr(pred.device)), "l1_loss_forward")
        ctx.save_for_backward(p, t, w)
        ctx.meta = (ldp, ldt, int(per_sample), pred.shape, rows)
        return loss

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        p, t, w = ctx.saved_tensors
        ldp, ldt, per_sample, shape, rows = ctx.meta
        if ctx.pre is not None:
            dp, gptr, gver = ctx.pre
            if g.data_ptr() == gptr and g._version == gver and g.numel() == 1:
                return dp.view(shape), None, None, None, None, None, None  # written by the forward launch
        total, cols = p.shape
        g = g.contiguous()
        dp = torch.empty(total, cols, dtype=_F32, device=p.device)
        check(lib.aimx_l1_loss_backward_padded(ptr(p), ldp, ptr(t), ldt, rows, total, cols, ptr(w), per_sample, ptr(g),
                                               ptr(dp), cols, stream_ptr(p.device)), "l1_loss_backward")
        return dp.view(shape), None, None, None, None, None, None


def l1_loss(pred, target, weights=None, per_sample=False, rows=None, accum=None, grad_of=None):
    """mean |pred - target| (per_sample=False, weights None: nn.L1Loss) or
    mean over samples of sum_t w_t |pred - target| (per_sample=True: WeightedL1Loss).
    rows=B: the loss of pred[:B] against target (B rows), with pred's remaining rows (the padding
    molecules of a static captured batch) getting a zero gradient in the same launch; equal to
    l1_loss(pred[:B], target) without autograd's slice-backward zero fill and copy.
    accum=(loss_sum f32[], nan_count i32[], steps i64[], scale): the train step's device-side
    bookkeeping in the same launch (loss_sum += loss * scale, nan_count += any(isnan(pred[:rows])),
    steps += 1; aimx_l1_loss_forward_accum).
    grad_of (with accum): the f32 scalar tensor the caller will pass to backward(); the forward
    launch then also writes the backward's gradient, and a backward with that same, unmodified
    tensor needs no launch (any other gradient runs the backward kernel as usual)."""
    if grad_of is not None and (accum is None or grad_of.dtype != _F32 or grad_of.numel() != 1):
        raise _lib.AimxError("aimx.l1_loss: grad_of is an f32 scalar tensor and needs accum")
    if accum is not None:
        ls, nc, st, _ = accum
        if ls.dtype != _F32 or nc.dtype != torch.int32 or st.dtype != torch.int64 or \
                ls.numel() != 1 or nc.numel() != 1 or st.numel() != 1:
            raise _lib.AimxError("aimx.l1_loss: accum = (f32 scalar, int32 scalar, int64 scalar, scale)")
    _lib.require_device(pred, target)
    if pred.dtype != _F32 or target.dtype != _F32:
        raise _lib.AimxError("aimx.l1_loss: pred and target must be fp32 tensors")
    if rows is None:
        if pred.shape != target.shape:
            raise _lib.AimxError("aimx.l1_loss: pred and target must have one shape")
    elif not (0 <= rows <= pred.shape[0] and target.shape[0] == rows and target.shape[1:] == pred.shape[1:]):
        raise _lib.AimxError("aimx.l1_loss: rows must be <= pred rows and equal target rows")
    return _L1Loss.apply(pred, target, weights, bool(per_sample), rows, accum, grad_of)


# ---------------------------------------------------------------------------------------------
# Fused post-pool head (gnn.py:252-258; MultiLayerPerceptron / LinearBlock layers.py:170-267)
# ---------------------------------------------------------------------------------------------
# widest ffn the fused head takes (head.hip kMaxF = 512)
HEAD_MAX_F = 512


class _Head(torch.autograd.Function):
    """Forward: one launch (aimx_head_forward). Backward: one launch for the input-gradient chain
    (aimx_head_backward) + one grouped launch for every weight and bias gradient."""

    @staticmethod
    def forward(ctx, spec, seed, x0, wp, bp, *rest):
        lib = _lib.load()
        dev = x0.device
        nb = spec["nb"]
        blocks = [rest[4 * i:4 * i + 4] for i in range(nb)]
        ws_, bs_, wo, bo = rest[4 * nb:4 * nb + 4]
        x0, ldx0 = _rows(x0)
        G, Hin = x0.shape
        F, T = wp.shape[0], wo.shape[0]
        drop = bool(spec["training"]) and spec["drop_p"] > 0 and seed is not None
        ar = Arena(dev)
        iy0 = ar.add(G, F)
        iv = [ar.add(G, F) for _ in range(nb)]
        ih = [ar.add(G, F) for _ in range(nb)]
        iz = [ar.add(G, F) for _ in range(nb)]
        icat = ar.add(G, 2 * F)
        buf, views = ar.alloc()
        masks = [torch.empty(G, F, dtype=torch.uint8, device=dev) for _ in range(nb)] if drop else []
        out = torch.empty(G, T, dtype=_F32, device=dev)
        h = _lib.Head()
        h.G, h.F, h.H_in, h.T = G, F, Hin, T
        h.nb, h.act, h.training = nb, spec["act"], int(drop)
        h.drop_p, h.seed = float(spec["drop_p"]) if drop else 0.0, ptr(seed) if drop else None
        h.x0, h.ldx0 = ptr(x0), ldx0
        wts = [wp.contiguous(), bp.contiguous()] + [t.contiguous() for t in rest]
        h.wp, h.bp = ptr(wts[0]), ptr(wts[1])
        for i in range(nb):
            w1, b1, w2, b2 = wts[2 + 4 * i:6 + 4 * i]
            h.w1[i], h.b1[i], h.w2[i], h.b2[i] = ptr(w1), ptr(b1), ptr(w2), ptr(b2)
            h.skip[i] = int(spec["skip"][i])
            h.v[i], h.hid[i], h.z[i] = ptr(views[iv[i]]), ptr(views[ih[i]]), ptr(views[iz[i]])
            h.mask[i] = ptr(masks[i]) if drop else None
        h.ws, h.bs, h.wo, h.bo = [ptr(t) for t in wts[2 + 4 * nb:6 + 4 * nb]]
        h.y0, h.cat = ptr(views[iy0]), ptr(views[icat])
        h.out, h.ldo = ptr(out), T
        h.sync, h.cluster = ptr(_lib.head_sync(dev)), spec["cluster"]
        # the 8-molecule kernels' transposed chain weights (0 bytes: the 16-molecule kernels)
        fwsb = lib.aimx_head_forward_workspace_bytes(h)
        fws = torch.empty(max(fwsb // 4, 4), dtype=_F32, device=dev) if fwsb else None
        h.fwd_ws, h.fwd_ws_bytes = (ptr(fws), fwsb) if fws is not None else (None, 0)
        check(lib.aimx_head_forward(h, stream_ptr(dev)), "head_forward")
        del fws
        ctx.spec, ctx.drop = spec, drop
        ctx.save_for_backward(x0, seed if drop else None, *wts)
        ctx.state = dict(buf=buf, views=views, iy0=iy0, iv=iv, ih=ih, iz=iz, icat=icat, masks=masks)
        return out

    @staticmethod
    def backward(ctx, d_out):
        lib = _lib.load()
        spec, st = ctx.spec, ctx.state
        x0, seed, *wts = ctx.saved_tensors
        nb = spec["nb"]
        dev = x0.device
        G, Hin = x0.shape
        F, T = wts[0].shape[0], wts[-2].shape[0]
        views = st["views"]
        d_out = d_out.contiguous()
        ar = Arena(dev)
        ids = ar.add(G, F)
        idz = [ar.add(G, F) for _ in range(nb)]
        idv = [ar.add(G, F) for _ in range(nb)]
        idy0 = ar.add(G, F)
        gbuf, gv = ar.alloc()
        d_x0 = torch.empty(G, Hin, dtype=_F32, device=dev)
        h = _lib.Head()
        h.G, h.F, h.H_in, h.T = G, F, Hin, T
        h.nb, h.act, h.training = nb, spec["act"], int(ctx.drop)
        h.drop_p, h.seed = float(spec["drop_p"]) if ctx.drop else 0.0, ptr(seed) if ctx.drop else None
        h.x0, h.ldx0 = ptr(x0), x0.stride(0)
        h.wp, h.bp = ptr(wts[0]), ptr(wts[1])
        for i in range(nb):
            w1, b1, w2, b2 = wts[2 + 4 * i:6 + 4 * i]
            h.w1[i], h.b1[i], h.w2[i], h.b2[i] = ptr(w1), ptr(b1), ptr(w2), ptr(b2)
            h.skip[i] = int(spec["skip"][i])
            h.v[i], h.hid[i], h.z[i] = ptr(views[st["iv"][i]]), ptr(views[st["ih"][i]]), ptr(views[st["iz"][i]])
            h.mask[i] = ptr(st["masks"][i]) if ctx.drop else None
        h.ws, h.bs, h.wo, h.bo = [ptr(t) for t in wts[2 + 4 * nb:6 + 4 * nb]]
        h.y0, h.cat = ptr(views[st["iy0"]]), ptr(views[st["icat"]])
        h.out, h.ldo = ptr(d_out), T  # unused by the backward (validity only)
        h.sync, h.cluster = ptr(_lib.head_sync(dev)), spec["cluster"]
        dg = _lib.HeadGrad()
        dg.d_out, dg.ld_dout = ptr(d_out), T
        dg.d_x0, dg.ld_dx0 = ptr(d_x0), Hin
        dg.ds, dg.dy0 = ptr(gv[ids]), ptr(gv[idy0])
        for i in range(nb):
            dg.dz[i], dg.dv[i] = ptr(gv[idz[i]]), ptr(gv[idv[i]])
        wsb = lib.aimx_head_backward_workspace_bytes(h)
        hws = torch.empty(max(wsb // 4, 1), dtype=_F32, device=dev)
        dg.workspace, dg.workspace_bytes = ptr(hws), wsb
        check(lib.aimx_head_backward(h, dg, stream_ptr(dev)), "head_backward")
        # every weight / bias gradient: dW = dY^T X over the G molecules, one grouped launch
        new = lambda *shape: torch.empty(*shape, dtype=_F32, device=dev)  # noqa: E731
        grads = [new(*t.shape) for t in wts]
        y = [views[st["iy0"]]] + [views[st["iz"][i]] for i in range(nb - 1)]
        probs = [(gv[idy0], x0, grads[0], grads[1])]
        for i in range(nb):
            probs.append((gv[idv[i]], y[i], grads[2 + 4 * i], grads[3 + 4 * i]))
            probs.append((gv[idz[i]], views[st["ih"][i]], grads[4 + 4 * i], grads[5 + 4 * i]))
        cat = views[st["icat"]]
        probs.append((gv[ids], views[st["iz"][nb - 1]], grads[2 + 4 * nb], grads[3 + 4 * nb]))
        probs.append((d_out, cat, grads[4 + 4 * nb], grads[5 + 4 * nb]))
        ws = wgrad_grouped(probs)
        del ws, gbuf, hws
        return (None, None, d_x0, *grads)


def head(x_pooled, wp, bp, blocks, ws, bs, wo, bo, *, act, drop_p=0.0, training=False, seed=None, skips=None):
    """out = output_layer([z | skip_transform(z)]), z = ffn(post_pooling_projection(x_pooled)) as the
    fused head (reference gnn.py:252-258). blocks: [(W1, b1, W2, b2)] of the LinearBlocks, skips:
    their use_skip flags. seed: int64 [1] device tensor when dropout is active."""
    _lib.require_device(x_pooled, wp, wo)
    nb = len(blocks)
    if not (1 <= nb <= _lib.HEAD_MAX_BLOCKS):
        raise _lib.AimxError("aimx.head: 1..8 LinearBlocks")
    kind = _lib.ACT_KIND[act] if isinstance(act, str) else int(act)
    drop = bool(training) and drop_p > 0
    if drop and seed is None:
        seed = torch.randint(0, 2 ** 62, (1,), device=x_pooled.device, dtype=torch.int64)
    spec = dict(nb=nb, act=kind, training=bool(training), drop_p=float(drop_p),
                skip=tuple(bool(s) for s in (skips or [False] * nb)), cluster=_lib.head_cluster(int(wp.shape[0])))
    flat = []
    for b in blocks:
        flat += list(b)
    return _Head.apply(spec, seed if drop else None, x_pooled, wp, bp, *flat, ws, bs, wo, bo)
