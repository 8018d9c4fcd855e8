"""Train step and epoch on the MI355X path — the reference trainer's loop (A18) made graph-replayable.

Reference: src/training/trainer.py:102-183 (_training_epoch): per batch
    zero_grad(set_to_none) -> model(7 args) -> isnan check -> criterion -> backward
    -> clip_grad_norm_(1.0) -> optimizer.step() -> loss.item() * batch_size
and, under DDP, one all-reduce of (loss sum, count) per epoch.

Here the same step runs either eagerly (`train_step`) or as captured HIP graphs (`GraphedTrainStep`)
over static padded batches (aimx.data.pad_collated / the native BatchFeeder padding): the first
call captures forward + loss + backward (+ the bucketed RCCL gradient all-reduce overlapped with
the backward when world > 1) + fused clip + Adam; every later batch is copied into the static
inputs and replayed. The per-step `loss.item()` and the NaN check of the reference are kept on the
device (a running loss sum and a NaN counter) and read once per epoch, so the loop never
synchronises the host per step.
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch
import torch.distributed as dist

from . import _lib


def _real_rows(batch):
    """Real (non-padding) molecules of a batch: padded batches carry real_graphs."""
    return int(getattr(batch, "real_graphs", batch.num_graphs))


def train_step(model, batch, criterion, optimizer, sync=None, n_real=None):
    """One eager step (trainer.py:128-168). Returns (loss tensor, nan flag tensor) on the device."""
    B = _real_rows(batch) if n_real is None else n_real
    optimizer.zero_grad(set_to_none=True)
    out, _, _ = model(*batch.model_args())
    nan = torch.isnan(out[:B]).any()
    loss = criterion(out[:B], batch.targets[:B])
    loss.backward()
    if sync is not None:
        sync.finish()
    optimizer.step()  # FusedAdam(max_grad_norm=1.0) == clip_grad_norm_(1.0) + Adam
    return loss.detach(), nan


def _snapshot(model, optimizer, dev):
    """Parameters, optimizer state and the dropout seed counters before GraphedTrainStep's warm-up."""
    from . import ops
    ops._seed_state(model, dev)  # the model's dropout counter exists before the warm-up draws from it
    params = [(p, p.detach().clone()) for p in model.parameters()]
    seeds = [(m._aimx_seed_state, m._aimx_seed_state.clone()) for m in model.modules()
             if torch.is_tensor(getattr(m, "_aimx_seed_state", None))]
    state = {p: {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
             for p, st in optimizer.state.items()}
    step_t = getattr(optimizer, "_step_t", None)
    return params, seeds, state, step_t.clone() if torch.is_tensor(step_t) else None


@torch.no_grad()
def _restore(saved, optimizer):
    """Put back what _snapshot saw, in place (the graphs hold these tensors' addresses). State the
    warm-up created (Adam's moments and step counts) goes back to its initial zeros."""
    params, seeds, state, step_t = saved
    for p, v in params:
        p.copy_(v)
    for t, v in seeds:
        t.copy_(v)
    for p, st in optimizer.state.items():
        old = state.get(p, {})
        for k, v in list(st.items()):
            if torch.is_tensor(v):
                if torch.is_tensor(old.get(k)):
                    v.copy_(old[k])
                else:
                    v.zero_()
            else:
                st[k] = old.get(k, type(v)(0) if isinstance(v, (int, float)) else v)
    cur = getattr(optimizer, "_step_t", None)
    if torch.is_tensor(cur):
        if step_t is not None and step_t.numel() <= cur.numel():
            cur.zero_()
            cur[: step_t.numel()].copy_(step_t)
        else:
            cur.zero_()


# test hook (tests/test_gpu_ddp.py sets it inside a rank process): GraphedTrainStep's "capture"
# attempt raises as a failing RCCL capture would, to exercise the split fallback on any box
INJECT_CAPTURE_FAILURE = False


class GraphedTrainStep:
    """The train step captured as HIP graphs on a static padded batch (see module docstring).

    Every replayed batch must have the same number of real molecules B (rows >= B of the
    per-molecule outputs are padding and excluded from the loss); a batch with a captured layout
    (same padded atom / edge / molecule counts and task count) is replayed. Without a data-parallel
    sync up to `max_layouts` layouts are captured, each on first sight (or ahead of time by
    prepare()): batches padded to a few atom-count buckets (bench.py pads to 256-atom buckets) then
    carry little padding each. Any other batch (a feeder's rare over-capacity batch, handed out
    unpadded) runs the same step eagerly on the same parameters, gradients, optimizer state and
    loss accumulators. optimizer must be capturable
    (FusedAdam). Construction runs `warmup` real steps on example_batch (allocator pools, plans,
    optimizer state, communicators) and then rewinds the parameters, the optimizer state and the
    dropout counter, so the first call is the reference loop's first step.

    Data-parallel modes (`sync`: a utils.distributed.GradientSync; `ddp_graph` picks one):
      "capture" (default over RCCL): ONE graph holds forward, backward, the bucketed RCCL
          all-reduces (issued by the gradient hooks as their buckets fill, on RCCL's stream, so they
          overlap the rest of the backward — DDP's reducer, reference runner.py:703-707), the
          averaging, clip and Adam. Needs sync.capturable (overlap on, nccl backend). If the
          capture raises on any rank, every rank falls back to "split".
      "split": forward+backward graph, then the all-reduce eagerly, then a clip+Adam graph (the
          only choice for gloo, whose collectives run on the host).
    """

    def __init__(self, model, criterion, optimizer, example_batch, n_real=None, sync=None, warmup=3,
                 ddp_graph=None, inject_capture_failure=None, max_layouts=1):
        # test hook (tests/test_gpu_ddp.py): make the "capture" attempt raise as a failing RCCL build
        # would, to exercise the split fallback on any box
        if inject_capture_failure is None:
            inject_capture_failure = INJECT_CAPTURE_FAILURE
        self.capture_error = None
        self.model, self.criterion, self.optimizer, self.sync = model, criterion, optimizer, sync
        self.warmup = warmup
        model._aimx_autograph_off = True  # this step captures the model itself (aimx.autograph stays off)
        self.B = _real_rows(example_batch) if n_real is None else int(n_real)
        dev = example_batch._blob.device
        self.dev = dev
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
        self.nan_count = torch.zeros((), dtype=torch.int32, device=dev)
        self.steps = torch.zeros((), dtype=torch.int64, device=dev)
        one = torch.ones((), dtype=torch.float32, device=dev)
        padded = getattr(criterion, "padded", None)
        B = self.B
        self.eager_steps = 0

        def fwd_bwd(batch):
            # the post-pool head runs on the B real molecules only (their rows are the loss's; the
            # padding molecules' outputs are never read): GNN._aimx_head_rows
            model.__dict__["_aimx_head_rows"] = B
            try:
                out, _, _ = model(*batch.model_args())
            finally:
                model.__dict__.pop("_aimx_head_rows", None)
            if padded is not None:
                # fused L1: the padding rows' zero gradient in the loss's backward launch, and the
                # step's loss sum / NaN flag / step count in its forward launch
                loss = padded(out, batch.targets[:B], B,
                              accum=(self.loss_sum, self.nan_count, self.steps, float(B)), grad_of=one)
            else:
                loss = criterion(out[:B], batch.targets[:B])
            loss.backward(one)  # d loss = 1 from a resident tensor (no per-step fill launch)
            if padded is None:
                self.loss_sum.add_(loss.detach() * B)
                self.nan_count.add_(torch.isnan(out[:B]).any().to(torch.int32))
                self.steps.add_(1)

        self._fwd_bwd = fwd_bwd
        mode = ddp_graph or "capture"
        if mode not in ("capture", "split"):
            raise ValueError(f"ddp_graph must be 'capture' or 'split', not {mode!r}")
        if sync is None or not sync.active:
            mode = "single"
        elif mode == "capture" and not sync.capturable:
            mode = "split"
        # more than one captured layout only without a data-parallel sync: a rank meeting a new layout
        # would capture (warm-up all-reduces) while its peers replay, and split mode's clip + Adam
        # graph reads the one set of gradient tensors the first capture made
        self.max_layouts = max(1, int(max_layouts)) if mode == "single" else 1
        self._graphs = {}
        self.mode = mode
        self._capture(example_batch, inject_capture_failure)
        self.reset_stats()

    def _capture(self, example_batch, inject_capture_failure=False):
        """Warm up on `example_batch` (real steps), capture the step on a static copy of it and rewind.
        The captured graphs join self._graphs under the batch's layout and become the current ones."""
        model, optimizer, sync, dev, mode = self.model, self.optimizer, self.sync, self.dev, self.mode
        static = example_batch.clone()
        fwd_bwd = self._fwd_bwd
        # the warm-up steps below really train (optimizer state, dropout counter): their starting
        # state is put back after the capture, so the next step is the loop's next step
        saved = _snapshot(model, optimizer, dev)
        stats = [t.clone() for t in (self.loss_sum, self.nan_count, self.steps)]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up: allocator pools, plans, optimizer state, RCCL comms
            for _ in range(self.warmup):
                optimizer.zero_grad(set_to_none=True)
                fwd_bwd(static)
                if sync is not None:
                    sync.finish()
                optimizer.step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        # single mode: each layout's graph holds its own gradient tensors (allocated in its capture,
        # in its private pool) and the Adam step that reads them
        optimizer.zero_grad(set_to_none=True)
        g1 = torch.cuda.CUDAGraph()
        g2 = None
        if mode == "single":
            with torch.cuda.graph(g1):
                fwd_bwd(static)
                optimizer.step()
        elif mode == "capture":
            ok = True
            err = None
            if dist.is_initialized():
                dist.barrier()
                torch.cuda.synchronize(dev)
            try:
                # thread_local: RCCL's watchdog thread may query events while this thread captures
                with torch.cuda.graph(g1, capture_error_mode="thread_local"):
                    fwd_bwd(static)
                    sync.finish()
                    if inject_capture_failure:
                        raise RuntimeError("injected capture failure (test hook)")
                    optimizer.step()
            except RuntimeError as e:  # depends on the RCCL build (and the test hook)
                ok, err = False, e
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag.item()) == 0:
                import sys
                print(f"aimx.train: RCCL all-reduce capture failed ({err}); using split graphs", file=sys.stderr)
                self.capture_error = str(err) if err is not None else "failed on another rank"
                sync._reset()
                optimizer.zero_grad(set_to_none=True)
                g1 = torch.cuda.CUDAGraph()
                mode = "split"
        if mode == "split":
            g2 = torch.cuda.CUDAGraph()
            hooks, sync._hooks = sync._hooks, []  # the eager all-reduce runs between the graphs
            for h in hooks:
                h.remove()
            sync.overlap = False
            with torch.cuda.graph(g1):
                fwd_bwd(static)
            with torch.cuda.graph(g2):
                optimizer.step()
        self.mode = mode
        _restore(saved, optimizer)
        with torch.no_grad():  # ... and the warm-up steps' loss sum, NaN count and step count
            for t, v in zip((self.loss_sum, self.nan_count, self.steps), stats):
                t.copy_(v)
        self._graphs[tuple(static._layout)] = (static, g1, g2)
        self.static, self.g1, self.g2 = static, g1, g2

    def prepare(self, batches):
        """Capture every new layout among `batches` now (up to max_layouts), so that no capture
        falls inside a timed loop; returns the number of layouts held."""
        for b in batches:
            key = tuple(b._layout)
            if key not in self._graphs and len(self._graphs) < self.max_layouts:
                self._capture(b)
        return len(self._graphs)

    @property
    def layouts(self):
        """Captured layouts (static batch shapes) so far."""
        return len(self._graphs)

    def reset_stats(self):
        self.loss_sum.zero_()
        self.nan_count.zero_()
        self.steps.zero_()

    def __call__(self, batch=None):
        """Copy `batch` (a DeviceBatch of a captured layout) into its static inputs and replay. A batch
        of a new layout is captured first while fewer than max_layouts are held, else run eagerly."""
        if batch is not None:
            n_real = _real_rows(batch)
            if n_real != self.B:  # e.g. a trailing partial batch: padding rows would enter the loss
                raise ValueError(f"GraphedTrainStep: batch has {n_real} real molecules, the captured step "
                                 f"takes exactly {self.B} (run partial batches through train_step)")
            if batch._layout != self.static._layout:
                got = self._graphs.get(tuple(batch._layout))
                if got is None and len(self._graphs) < self.max_layouts:
                    self._capture(batch)
                    got = self._graphs[tuple(batch._layout)]
                if got is None:
                    self._eager(batch)
                    return
                self.static, self.g1, self.g2 = got
            self.static.copy_(batch)
        self.g1.replay()
        if self.g2 is not None:
            self.sync.finish()
            self.g2.replay()

    def _eager(self, batch):
        """The captured step, run eagerly on a batch of another layout. The gradients are zeroed in
        place (not set to None): the parameters keep the .grad tensors the graphs write and the
        optimizer reads; with a GradientSync the same bucketed all-reduces run (hooks, finish)."""
        self.eager_steps += 1
        self.optimizer.zero_grad(set_to_none=False)
        self._fwd_bwd(batch)
        if self.sync is not None:
            self.sync.finish()
        self.optimizer.step()


def train_epoch(model, batches: Iterable, criterion, optimizer, device, sync=None, graphed: Optional[
        GraphedTrainStep] = None):
    """One epoch (trainer.py:102-183). batches: DeviceBatch objects (e.g. from aimx.feed.BatchFeeder).
    With `graphed`, every batch is replayed through the captured step (static layout required).
    Returns (epoch mean loss over molecules, DDP-reduced like the reference, number of NaN steps)."""
    dev = torch.device(device)
    loss_sum = torch.zeros((), dtype=torch.float64, device=dev)
    count = 0
    nans = torch.zeros((), dtype=torch.int64, device=dev)
    if graphed is not None:
        graphed.reset_stats()
    for batch in batches:
        if graphed is not None:
            graphed(batch)
            count += graphed.B
            continue
        B = _real_rows(batch)
        loss, nan = train_step(model, batch, criterion, optimizer, sync, B)
        loss_sum += loss.double() * B
        nans += nan.to(torch.int64)
        count += B
    if graphed is not None:
        loss_sum = graphed.loss_sum.double()
        nans = graphed.nan_count.to(torch.int64)
    # the clustered head's sticky timeout word (include/aimx.h AimxHead.sync) rides along in the
    # epoch's one collective, so every rank sees any rank's timeout and all of them raise together
    # (a rank raising alone would leave the others blocked in the next collective)
    t = torch.stack([loss_sum, torch.tensor(float(count), dtype=torch.float64, device=dev), nans.double(),
                     _lib.head_sync_flag(dev)])
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t)
    s, c, n, tmo = t.tolist()
    if tmo != 0:
        raise RuntimeError("aimx: a clustered head launch timed out waiting for its cluster this epoch "
                           "(results invalid; set aimx._lib.HEAD_CLUSTER_FORCE = 1)")
    return (s / c if c > 0 else 0.0), int(n)


def main(argv=None):
    """QM9 training on the committed QM9-val graph asset (13,373 molecules): 90/10 split, one target
    (z-scored), the reference defaults (hidden 256, 3 hops, attention pool, L1, Adam 2.5e-4,
    clip 1.0), native feed, graphed steps. One process per GPU under torchrun (disjoint index
    shards per rank, gradients all-reduced by GradientSync over RCCL)."""
    import argparse
    import os
    import time

    import numpy as np

    from models import GNN, L1Loss
    from utils.distributed import GradientSync

    from . import data as adata
    from . import feed
    from .optim import FusedAdam
    from .synth import QM9Asset

    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--target", type=int, default=0)
    ap.add_argument("--lr", type=float, default=2.5e-4)
    ap.add_argument("--limit", type=int, default=0, help="use only the first N molecules (0: all)")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    torch.manual_seed(a.seed)
    asset = QM9Asset()
    n = len(asset) if a.limit <= 0 else min(a.limit, len(asset))
    rng = np.random.default_rng(a.seed)
    perm = rng.permutation(n)
    n_tr = int(0.9 * n)
    tr_idx, va_idx = perm[:n_tr], perm[n_tr:]
    y = asset.targets[:, a.target:a.target + 1].astype(np.float32)
    mu, sd = float(y[tr_idx].mean()), float(y[tr_idx].std() + 1e-6)
    store = feed.HostStore.from_arrays(asset.atom_off, asset.bond_off, np.stack([asset.bi, asset.bj], 1), asset.feats,
                                       (y - mu) / sd, asset.total_charge, precompute_hops=a.hops, threads=4)
    fs = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}
    model = GNN(fs, a.hidden, 1, num_shells=a.hops).to(dev).train()
    crit = L1Loss()
    opt = FusedAdam(model.parameters(), lr=a.lr, max_grad_norm=1.0)
    sync = GradientSync(model.parameters(), unused=model.unused_parameters()) if world > 1 else None
    B = a.batch
    shard = tr_idx[rank::world]  # disjoint per rank (DistributedSampler semantics)
    steps = len(shard) // B
    pad = not a.eager
    n_max = e_max = pm = 0
    if pad:
        n_max, e_max, pm = feed.static_capacity(feed.HostCollator(a.hops, 2), store,
                                                [shard[rng.permutation(len(shard))[:B]] for _ in range(256)])

    def epoch_batches(ep):
        p = np.random.default_rng(a.seed * 1000 + ep).permutation(len(shard))
        idx = [shard[p[i * B:(i + 1) * B]] for i in range(steps)]
        # ring: the graphed step copies each batch into its static inputs (feed.BatchFeeder)
        return feed.BatchFeeder(store, iter(idx), a.hops, dev, depth=3, threads=4, n_max=n_max, e_max=e_max,
                                pad_mols=pm, ring=pad)

    graphed = None
    for ep in range(a.epochs):
        t0 = time.perf_counter()
        batches = epoch_batches(ep)
        if pad and graphed is None:
            first = next(batches)
            graphed = GraphedTrainStep(model, crit, opt, first, n_real=B, sync=sync)
            graphed.reset_stats()
            import itertools
            batches = itertools.chain([first], batches)
        loss, nans = train_epoch(model, batches, crit, opt, dev, sync=sync, graphed=graphed)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # validation MAE (eager, eval mode), in target units
        model.eval()
        va = va_idx[rank::world]
        col = feed.HostCollator(a.hops, 2)
        err = torch.zeros((), dtype=torch.float64, device=dev)
        cnt = 0
        with torch.no_grad():
            for i in range(0, len(va), B):
                blob, layout, gr, nr, _ = col.collate_blob(store, va[i:i + B], pinned=True)
                vb = __import__("aimx.data", fromlist=["DeviceBatch"]).DeviceBatch.from_blob(
                    blob.to(dev, non_blocking=True), layout, gr, nr)
                out, _, _ = model(*vb.model_args())
                err += (out - vb.targets).abs().sum().double() * sd
                cnt += out.numel()
        t = torch.stack([err, torch.tensor(float(cnt), dtype=torch.float64, device=dev)])
        if world > 1:
            dist.all_reduce(t)
        model.train()
        if rank == 0:
            print(f"epoch {ep + 1}: train L1 {loss:.4f} (z-scored), val MAE {t[0].item() / t[1].item():.4f}, "
                  f"NaN steps {nans}, {steps * B * world / dt:.0f} mol/s incl. feed", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
