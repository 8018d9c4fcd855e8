"""Drop-in autograph: the unchanged eager trainer's GNN forward and backward replayed as HIP graphs.

The reference trainer (src/training/trainer.py:151-164) runs every step eagerly:
    output, _, _ = model(*batch); loss = criterion(output, y); loss.backward(); optimizer.step()
Eagerly, the c2 step is bound by the host (~60 operator calls through Python and ctypes per
step, ~2 ms) rather than by the ~0.9 ms of device work. By default (AIMX_AUTOGRAPH=0 or
`enable(model, False)` turns it off), `GNN.forward` in training mode instead:

  * pads the batch into the static inputs of a shape bucket — the smallest live one with the same
    molecule count and room for the batch's atoms (plus one slack atom) and edges; a new bucket
    takes ~6 % headroom, atoms rounded up to a multiple of 512 and edges to 4096; a bucket serves a
    batch only while its padding molecules stay within 96 atoms — in ONE launch (`aimx_pad_batch`:
    slack atoms form padding molecules (at least 8, ~64 atoms each down to 80 % occupancy), slack
    edges are self-pairs over them, the layout of aimx.data.pad_collated, so no real molecule's
    values change);
  * replays the bucket's forward graph and returns the real molecules' rows of the output through
    an autograd node whose backward copies the incoming gradient into the static gradient buffer
    and replays the bucket's backward graph;
  * hands the parameters their gradients as the bucket's static gradient tensors (assigned when
    `.grad` is None — `zero_grad(set_to_none=True)`, PyTorch's default; accumulated otherwise).

By default it applies to batches whose atoms x hidden width is at most MAX_WORK (device-bound
larger steps run eagerly, measured faster); `enable(model, True)` forces it for any size.

A bucket is captured on first use (warm-up on a side stream, then the forward graph and the
backward graph, each in its own memory pool so that no replay overwrites the other's live
tensors). The eager path
is used instead when a graph cannot reproduce eager semantics: grad disabled or eval mode,
stereochemistry inputs, a batch without edges, stream capture already active (GraphedTrainStep),
or forward hooks on a submodule (a replay fires none). Under an initialised process group
(DistributedDataParallel's reducer hooks every gradient accumulator, reference runner.py:703-707)
or with gradient hooks on the parameters, the replayed gradients are handed out through autograd
(_ReplayGrads) so the accumulators, their hooks and DDP's bucketed all-reduce see every one of
them. Parameters replaced since the capture (new
Parameter objects or moved storage) re-capture the bucket, and the autocast state is part of the
bucket key (a capture bakes in the GEMMs' bf16 or fp32 operands). The attention weights and partial charges come back as detached copies.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import AimxError, check, ptr, stream_ptr

ATOM_QUANTUM = 512
EDGE_QUANTUM = 4096
PAD_MOLS = 8          # fewest padding molecules of a bucket
PAD_ATOMS = 64        # ... sized for batches of >= (1 - MAX_SLACK) * Np atoms to keep each <= PAD_ATOMS
MAX_SLACK = 0.2
PAD_ATOMS_MAX = 96    # a bucket serves a batch only if its padding molecules stay within this (< 128)
MAX_BUCKETS = 4
_FEATURE_KEYS = ("atom_type", "hydrogen_count", "degree", "hybridization")


def enable(model, on=True):
    """Turn the autograph on (or off) for one GNN, whatever AIMX_AUTOGRAPH says."""
    model._aimx_autograph_on = bool(on)
    return model


# The replay pays off while the eager step is bound by the host's launches (c2: 2.2 ms eager vs
# 0.92 ms replayed); once the device work per step outgrows them, the bucket's padding and the per-step
# CSR build cost more than the launches saved (c4: 4.00 vs 3.29 ms eager, c5: 5.64 vs 5.14 ms;
# profiles/r02_bench_c4.json, r02_bench_c5.json). Gate: atoms x hidden width of the batch (c2 / c3
# 2.4 M, c4 / c5 10.4 M); an explicit enable(model, True) replays whatever the size.
MAX_WORK = 6_000_000


def wanted(model, args):
    on = getattr(model, "_aimx_autograph_on", None)
    explicit = on is not None
    if on is None:
        on = os.environ.get("AIMX_AUTOGRAPH", "1") != "0"
    if not on or getattr(model, "_aimx_autograph_off", False):
        return False
    if not (model.training and torch.is_grad_enabled()) or torch.cuda.is_current_stream_capturing():
        return False
    feats, edges, batch, charges, tet, cis, trans = args
    if not explicit and batch.shape[0] * int(getattr(model, "hidden_dim", 0)) > MAX_WORK:
        return False
    if edges.numel() == 0 or edges.dim() != 2 or edges.shape[1] != 2 or edges.dtype != torch.int64:
        return False
    if model.use_stereochemistry and (tet.numel() or cis.numel() or trans.numel()):
        return False
    if charges.dtype != torch.float32 or batch.dtype != torch.int64 or charges.dim() != 1:
        return False
    if any(feats[k].dtype != torch.int64 or feats[k].dim() != 1 for k in _FEATURE_KEYS):
        return False
    st = _state(model)
    return not st.forward_hooked(model)


def _dist_initialized():
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()
    except Exception:  # pragma: no cover
        return False


def _through_autograd(model):
    """Hand the gradients out through autograd (the parameters' AccumulateGrad nodes) instead of
    assigning .grad: whenever something may be watching them — a process group is initialised
    (DistributedDataParallel's reducer hooks every gradient accumulator, reference runner.py:703-707,
    and averages the buckets as they become ready), or a parameter carries gradient hooks. (Under
    DDP with the model's own sync, run() takes _ReplayDDP instead unless other hooks exist.)"""
    sync = model.__dict__.get("_aimx_sync")
    return _dist_initialized() or _state(model).grad_hooked(model, sync.hook_ids if sync is not None else ())


# Module-structure generation: bumped whenever a parameter or a submodule is registered anywhere
# (nn.Module.__setattr__ / register_parameter / load_state_dict(assign=True) / a swapped submodule)
# and by GNN._apply (.to(), .cuda(): parameters in new storage). The per-step checks below read a
# cached parameter / module list while it is unchanged instead of walking the module tree (the walks
# cost ~0.4 ms of host time per step — more than a c2 step's replay).
_GEN = [0]


def _bump(*_):
    _GEN[0] += 1


def bump_structure():
    """Invalidate every model's cached parameter / module lists (GNN._apply calls it)."""
    _bump()


torch.nn.modules.module.register_module_parameter_registration_hook(_bump)
torch.nn.modules.module.register_module_module_registration_hook(_bump)


class _State:
    def __init__(self):
        self.buckets = {}
        self.order = []
        self.anchor = None
        self.gen = -1
        self.params = self.modules = None

    def structure(self, model):
        """(parameters, submodules, parameter identity key), rebuilt only when _GEN moved."""
        if self.gen != _GEN[0]:
            self.params = list(model.parameters())
            self.modules = [m for m in model.modules() if m is not model]
            self.gen = _GEN[0]
        return self

    def forward_hooked(self, model):
        """Forward hooks on a submodule: a replay cannot fire them (the eager path runs instead)."""
        return any(m._forward_hooks or m._forward_pre_hooks for m in self.structure(model).modules)

    def grad_hooked(self, model, ignore=()):
        """Gradient hooks on a parameter (other than the handles in `ignore`: the model's own
        gradient sync): the replay then hands its gradients out through autograd."""
        for p in self.structure(model).params:
            for d in (p._post_accumulate_grad_hooks, p._backward_hooks):
                if d and any(k not in ignore for k in d):
                    return True
        return False


def _state(model):
    st = model.__dict__.get("_aimx_autograph_state")
    if st is None:
        st = _State()
        model.__dict__["_aimx_autograph_state"] = st
    return st


def _round_up(x, q):
    return (x + q - 1) // q * q


def pad_mols_for(Np):
    """Padding molecules of a bucket of Np atoms (aimx.data.pad_mols_for for batches down to
    (1 - MAX_SLACK) * Np atoms)."""
    from .data import pad_mols_for as pm
    return pm(Np, int((1 - MAX_SLACK) * Np), PAD_ATOMS, PAD_MOLS)


def _param_key(model):
    """Identity and storage of the model's live parameters: a replaced Parameter object
    (load_state_dict(assign=True), a swapped submodule) or moved storage re-captures the bucket.
    The parameter list is cached (rebuilt when _GEN moves), the storage pointers are read every
    call: `p.data = ...` (vector_to_parameters, an EMA / SWA swap) or a submodule's .to() / .half()
    moves a parameter's storage without registering anything."""
    return tuple((id(p), p.data_ptr()) for p in _state(model).structure(model).params)


def _amp_key():
    """The autocast state a capture bakes in (the GEMMs pick bf16 or fp32 operands at capture)."""
    on = torch.is_autocast_enabled("cuda")
    return (on, torch.get_autocast_dtype("cuda") if on else None)


class _Bucket:
    """Static padded inputs, the captured forward / backward graphs and their static outputs."""

    def __init__(self, model, Np, Ep, G, dev):
        i64 = torch.int64
        self.Np, self.Ep, self.G, self.dev = Np, Ep, G, dev
        self.feat = torch.zeros(4, Np, dtype=i64, device=dev)
        self.edges = torch.zeros(Ep, 2, dtype=i64, device=dev)
        self.batch = torch.zeros(Np, dtype=i64, device=dev)
        self.pad_mols = pad_mols_for(Np)
        self.charges = torch.zeros(G + self.pad_mols, dtype=torch.float32, device=dev)
        self.empty4 = torch.empty(0, 4, dtype=i64, device=dev)
        self.empty2 = torch.empty(0, 2, dtype=i64, device=dev)
        a = _lib.PadBatch()
        a.out_feat, a.out_edges, a.out_batch, a.out_charges = ptr(self.feat), ptr(self.edges), ptr(self.batch), \
            ptr(self.charges)
        a.Np, a.Ep, a.pad_mols = Np, Ep, self.pad_mols
        self.pad = a
        self.params = list(_state(model).structure(model).params)
        self.param_key = _param_key(model)
        self.gen = 0        # forward replays so far
        self.done = -1      # generation whose backward has run

    def static_args(self):
        return ({k: self.feat[i] for i, k in enumerate(_FEATURE_KEYS)}, self.edges, self.batch, self.charges,
                self.empty4, self.empty2, self.empty2)

    def fill(self, feats, edges, batch, charges):
        a = self.pad
        for i, k in enumerate(_FEATURE_KEYS):
            t = feats[k]
            a.feat[i] = t.data_ptr()
            a.feat_stride[i] = t.stride(0)
        a.edges, a.edge_s0, a.edge_s1 = edges.data_ptr(), edges.stride(0), edges.stride(1)
        a.batch, a.batch_stride = batch.data_ptr(), batch.stride(0)
        a.charges, a.charge_stride = charges.data_ptr(), charges.stride(0)
        a.N, a.E, a.G = batch.shape[0], edges.shape[0], charges.shape[0]
        check(_lib.load().aimx_pad_batch(ctypes.byref(a), stream_ptr(self.dev)), "autograph pad_batch")

    def capture(self, model, warmup=2):
        # The warm-up and captured backward passes compute the gradients with autograd.grad, not
        # .backward(), and with respect to stand-ins of the parameters (_aliased): no AccumulateGrad
        # node runs or receives a gradient, so no hook on the parameters fires for them (DDP's
        # reducer would take each for a real backward), no .grad is touched, and the engine never
        # synchronises with the stream an accumulator was made on (DDP makes them at construction,
        # on the default stream, which a capture must not wait on)
        params = self.params
        live = [p for p in params if p.requires_grad]
        args = self.static_args()
        cur = torch.cuda.current_stream(self.dev)
        side = torch.cuda.Stream(device=self.dev)
        side.wait_stream(cur)
        # the post-pool head runs on the G real molecules only (GNN._aimx_head_rows): the replay
        # hands out outs[0][:G], the padding molecules' rows are never read
        model.__dict__["_aimx_head_rows"] = self.G
        try:
            self._capture(model, warmup, params, live, args, cur, side)
        finally:
            model.__dict__.pop("_aimx_head_rows", None)

    def _capture(self, model, warmup, params, live, args, cur, side):
        with torch.cuda.stream(side):  # warm-up: plans, workspaces, allocator pools, seed state
            for _ in range(warmup):
                with _aliased(model, live) as al:
                    out = model._aimx_forward(*args)[0]
                    torch.autograd.grad(out, [al[id(p)] for p in live], torch.zeros_like(out), allow_unused=True)
                # drop the warm-up graph before the capture: alive, its nodes would stay bound to
                # this side stream while the captured backward runs on the capture stream
                del out, al
        cur.wait_stream(side)
        torch.cuda.synchronize(self.dev)
        # under a process group, another thread (ProcessGroupNCCL's watchdog) may query its events
        # while the capture is open: a global-mode capture would be invalidated by that query, a
        # thread-local one only watches this thread (as GraphedTrainStep captures, train.py)
        mode = "thread_local" if _dist_initialized() else "global"
        self.g_fwd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fwd, capture_error_mode=mode):
            with _aliased(model, live) as al:
                self.outs = model._aimx_forward(*args)
        stand_ins = [al[id(p)] for p in live]
        del al
        self.gout = torch.zeros_like(self.outs[0])
        # the backward graph gets its own memory pool: in a shared one, the gradient tensors it
        # leaves behind could sit in blocks the forward graph used (and frees) for temporaries,
        # and the next forward replay would overwrite the caller's .grad
        self.g_bwd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_bwd, capture_error_mode=mode):
            gs = torch.autograd.grad(self.outs[0], stand_ins, self.gout, allow_unused=True)
        del stand_ins
        by_id = {id(p): g for p, g in zip(live, gs)}
        self.grads = [by_id.get(id(p)) for p in params]
        self.outs = tuple(o.detach() if o is not None else None for o in self.outs)


class _aliased:
    """Every live parameter swapped, in its modules' _parameters, for a non-leaf alias
    (p.view_as(p): same storage, made on the current stream) while a warm-up or captured pass
    builds its graph; the parameters are put back on exit. Gradients taken with respect to the
    aliases stop at their view nodes, short of the parameters' AccumulateGrad nodes."""

    def __init__(self, model, live):
        self.model, self.live = model, live

    def __enter__(self):
        ids = {id(p) for p in self.live}
        self.saved = [(m, n, p) for m in self.model.modules() for n, p in m._parameters.items()
                      if p is not None and id(p) in ids]
        al = {id(p): p.view_as(p) for p in self.live}
        for m, n, p in self.saved:
            m._parameters[n] = al[id(p)]
        return al

    def __exit__(self, *exc):
        for m, n, p in self.saved:
            m._parameters[n] = p
        self.saved = None
        return False


class _Replay(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, bucket, G):
        ctx.bucket, ctx.G, ctx.gen = bucket, G, bucket.gen
        return bucket.outs[0][:G].clone()

    @staticmethod
    def backward(ctx, gout):
        b = ctx.bucket
        if b.gen != ctx.gen or b.done == ctx.gen:
            raise AimxError("aimx autograph: this output's saved state was overwritten by a later forward of the "
                            "same shape bucket (or its backward already ran); run one backward per forward, or "
                            "set AIMX_AUTOGRAPH=0")
        b.gout[:ctx.G].copy_(gout)
        _move_aliased_grads(b)
        b.g_bwd.replay()
        b.done = ctx.gen
        for p, sg in zip(b.params, b.grads):
            if sg is None:
                continue
            if p.grad is None:
                p.grad = sg                      # zero_grad(set_to_none=True): the fast path
            else:
                p.grad.add_(sg)
        return None, None, None


_RT_KEYS = __import__("itertools").count()


def _move_aliased_grads(b):
    """A .grad still sharing storage with its static gradient (handed out as the tensor itself or a
    view of it by an earlier step and not reset since: accumulation, DDP no_sync micro-batches)
    would be overwritten by the replay and then accumulated onto itself (2 g_new instead of
    g_old + g_new): move it out first."""
    for p, sg in zip(b.params, b.grads):
        if sg is not None and p.grad is not None and p.grad.untyped_storage().data_ptr() == \
                sg.untyped_storage().data_ptr():
            p.grad = p.grad.clone()


class _ReplayDDP(torch.autograd.Function):
    """_Replay under DistributedDataParallel with the model's own gradient sync
    (GNN._ddp_params_and_buffers_to_ignore): the anchor parameter, the one DDP's reducer keeps, gets
    its gradient through autograd (DDP's hooks and end-of-backward bookkeeping run on it); every
    other gradient is averaged across the ranks by the sync right after the backward replay (pack,
    one all-reduce per bucket, unpack) and handed to .grad as _Replay does."""

    @staticmethod
    def forward(ctx, anchor, bucket, G, sync, p_anchor):
        ctx.bucket, ctx.G, ctx.gen, ctx.sync, ctx.p_anchor = bucket, G, bucket.gen, sync, p_anchor
        return bucket.outs[0][:G].clone()

    @staticmethod
    def backward(ctx, gout):
        b, pa = ctx.bucket, ctx.p_anchor
        if b.gen != ctx.gen or b.done == ctx.gen:
            raise AimxError("aimx autograph: this output's saved state was overwritten by a later forward of the "
                            "same shape bucket (or its backward already ran); run one backward per forward, or "
                            "set AIMX_AUTOGRAPH=0")
        b.gout[:ctx.G].copy_(gout)
        _move_aliased_grads(b)
        b.g_bwd.replay()
        b.done = ctx.gen
        sync = ctx.sync
        fresh = all(p.grad is None for p, sg in zip(b.params, b.grads) if sg is not None and p is not pa)
        if fresh and sync.syncing():
            # the fast path (zero_grad(set_to_none=True), every backward synced): average the
            # replay's static gradients in place, then hand them out
            rt = b.__dict__.get("_rt_grads")
            if rt is None:  # the bucket's static gradients: the same tensors every replay
                rt = b._rt_grads = {id(p): sg for p, sg in zip(b.params, b.grads) if sg is not None and p is not pa}
                b._rt_key = next(_RT_KEYS)  # never reused (an id() could be, after the bucket is gone)
            sync.reduce_tensors(rt, key=b._rt_key)
        ga = None
        acc = {}
        for p, sg in zip(b.params, b.grads):
            if sg is None:
                continue
            if p is pa:
                ga = sg.clone()  # DDP's reducer averages this one (and may write into .grad)
            elif p.grad is None:
                p.grad = sg
            else:
                p.grad.add_(sg)
            if p is not pa:
                acc[id(p)] = p.grad
        if not fresh and sync.syncing():
            # accumulation (earlier micro-batches' gradients, e.g. under ddp.no_sync()): DDP averages
            # the ACCUMULATED gradient at the synced backward, so this sums first and averages after
            sync.reduce_tensors(acc)
        return None, None, None, None, ga


class _ReplayGrads(torch.autograd.Function):
    """_Replay for watched gradients (_through_autograd): the parameters with a gradient are inputs,
    and the backward replay's static gradients come back as their gradients, so autograd's
    AccumulateGrad nodes — and every hook on them, DDP's reducer included — see each one. (The
    engine clones a gradient the bucket still references, so each step's values stay the caller's.)"""

    @staticmethod
    def forward(ctx, anchor, bucket, G, *params):
        ctx.bucket, ctx.G, ctx.gen = bucket, G, bucket.gen
        return bucket.outs[0][:G].clone()

    @staticmethod
    def backward(ctx, gout):
        b = ctx.bucket
        if b.gen != ctx.gen or b.done == ctx.gen:
            raise AimxError("aimx autograph: this output's saved state was overwritten by a later forward of the "
                            "same shape bucket (or its backward already ran); run one backward per forward, or "
                            "set AIMX_AUTOGRAPH=0")
        b.gout[:ctx.G].copy_(gout)
        _move_aliased_grads(b)
        b.g_bwd.replay()
        b.done = ctx.gen
        # every .grad None (zero_grad(set_to_none=True), the default): fresh views of the static
        # gradients, which the AccumulateGrad nodes take as they are (the parameters' .grad then
        # alias the bucket's static gradients, as _Replay hands them out) instead of cloning each
        # one — 73 launches per step at c2. Otherwise the static tensors themselves: the engine
        # clones them, so accumulating onto an existing .grad never reads memory the next replay
        # overwrites.
        fresh = all(p.grad is None for p, sg in zip(b.params, b.grads) if sg is not None)
        return (None, None, None, *[sg.view_as(sg) if fresh else sg for sg in b.grads if sg is not None])


def _pick(st, N, E, G, dev, amp):
    """The smallest live bucket that holds this batch (same molecule count and autocast state, room
    for one slack atom and every edge, padding molecules within PAD_ATOMS_MAX), else a new one sized
    with ~6 % headroom so the batches of an epoch settle on one or two buckets."""
    best = None
    for key, b in st.buckets.items():
        if key[2] == G and key[3] == dev.index and key[4] == amp and key[0] > N and key[1] >= E and \
                key[0] - N <= pad_mols_for(key[0]) * PAD_ATOMS_MAX and \
                (best is None or key[0] + key[1] < best[0] + best[1]):
            best = key
    if best is not None:
        return best, False
    return (_round_up(int(1.06 * (N + 1)) + 1, ATOM_QUANTUM), _round_up(int(1.06 * E) + 1, EDGE_QUANTUM), G,
            dev.index, amp), True


def run(model, args):
    """GNN.forward through the bucket's graphs (see the module docstring)."""
    feats, edges, batch, charges = args[:4]
    N, E, G = batch.shape[0], edges.shape[0], charges.shape[0]
    dev = batch.device
    st = _state(model)
    key, fresh = _pick(st, N, E, G, dev, _amp_key())
    b = st.buckets.get(key)
    if b is not None and b.param_key != _param_key(model):
        st.buckets.pop(key)
        st.order.remove(key)
        b, fresh = None, True
    if fresh:
        if len(st.order) >= MAX_BUCKETS:
            st.buckets.pop(st.order.pop(0))
        b = _Bucket(model, key[0], key[1], G, dev)
    else:
        st.order.remove(key)
    st.order.append(key)  # least recently used first
    b.fill(feats, edges, batch, charges)
    if fresh:
        b.capture(model)
        st.buckets[key] = b
    b.g_fwd.replay()
    b.gen += 1
    if st.anchor is None or st.anchor.device != dev:
        st.anchor = torch.zeros((), device=dev, requires_grad=True)
    native = model._aimx_native_sync() if hasattr(model, "_aimx_native_sync") else None
    p_anchor = getattr(native, "anchor_param", None)
    if native is not None and p_anchor is not None and not st.grad_hooked(model, native.hook_ids):
        out = _ReplayDDP.apply(st.anchor, b, G, native, p_anchor)
    elif _through_autograd(model):
        out = _ReplayGrads.apply(st.anchor, b, G, *[p for p, sg in zip(b.params, b.grads) if sg is not None])
    else:
        out = _Replay.apply(st.anchor, b, G)
    return out, _atoms(b.outs[1], b.Np, N), _atoms(b.outs[2], b.Np, N)


def _atoms(t, Np, N):
    """The real atoms' part of a per-atom static output (atoms on its first or last dim), copied."""
    if t is None:
        return None
    if t.shape[-1] == Np:
        return t[..., :N].clone()
    return t[:N].clone()
