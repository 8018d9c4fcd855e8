"""Distributed utilities — drop-in for reference src/utils/distributed.py (12-228) plus the
DDP-equivalent gradient synchronisation the hot path needs.

The reference's helpers keep their names, arguments and rank-0 return conventions
(gather_*_to_rank0 return the gathered data on rank 0 and an empty result elsewhere). On ROCm the
"nccl" backend of torch.distributed is RCCL, which runs over xGMI inside an MI355X node.

GradientSync replaces DistributedDataParallel's reducer (reference runner.py:703-707) for the
hot loop: gradients are packed into flat fp32 buckets (<= bucket_mb each, reverse registration
order, i.e. roughly the order backward produces them), each bucket is all-reduced with ONE RCCL
call as soon as every gradient in it has been accumulated (post-accumulate-grad hooks), so the
collectives overlap the rest of the backward, and finish() waits, averages (DDP semantics:
sum / world_size) and writes the result back into .grad. Parameters whose gradient is still None
after backward (e.g. the reference's never-used long_range_projection) are reduced as zeros and
left None, as DDP(find_unused_parameters=True) leaves them. One process per GPU; molecules are
sharded across ranks, so this all-reduce is the only data-path collective.
"""
import pickle
from typing import Any, List

import numpy as np
import torch
import torch.distributed as dist


def _ready() -> bool:
    return dist.is_available() and dist.is_initialized()


def is_main_process() -> bool:
    """True on rank 0 or when torch.distributed is not initialised."""
    return (not _ready()) or dist.get_rank() == 0


def safe_get_rank() -> int:
    return dist.get_rank() if _ready() else 0


def get_world_size() -> int:
    return dist.get_world_size() if _ready() else 1


def gather_ndarray_to_rank0(arr: np.ndarray, device: str = "cpu") -> np.ndarray:
    """All ranks' arrays (possibly different lengths) concatenated on rank 0 (as float32, like the
    reference); other ranks get an empty array of the input dtype."""
    if not _ready():
        return arr
    local = torch.from_numpy(arr).float().to(device)
    n_local = torch.tensor([local.shape[0]], dtype=torch.long, device=device)
    world = dist.get_world_size()
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local)
    n_max = max(int(s.item()) for s in sizes)
    if local.shape[0] < n_max:
        pad = torch.zeros((n_max - local.shape[0],) + tuple(local.shape[1:]), device=device)
        local = torch.cat([local, pad], dim=0)
    parts = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(parts, local)
    if dist.get_rank() != 0:
        return np.array([], dtype=arr.dtype)
    return np.concatenate([p[: int(s.item())].cpu().numpy() for p, s in zip(parts, sizes)], axis=0)


def _gather_bytes(payload: bytes, device: str):
    world = dist.get_world_size()
    n_local = torch.tensor([len(payload)], dtype=torch.long, device=device)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local)
    n_max = max(int(s.item()) for s in sizes)
    buf = torch.zeros(n_max, dtype=torch.uint8, device=device)
    if payload:
        buf[: len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    parts = [torch.zeros(n_max, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(parts, buf)
    return [p[: int(s.item())].cpu().numpy().tobytes() for p, s in zip(parts, sizes)]


def gather_strings_to_rank0(local_list: List[str], device: str = "cpu") -> List[str]:
    """All ranks' string lists concatenated on rank 0 (rank order); [] elsewhere."""
    if not _ready():
        return local_list
    chunks = _gather_bytes(pickle.dumps(local_list), device)
    if dist.get_rank() != 0:
        return []
    out: List[str] = []
    for c in chunks:
        out.extend(pickle.loads(c))
    return out


def broadcast_object(obj: Any, src_rank: int = 0, device: str = "cpu") -> Any:
    """Pickle-broadcast `obj` from `src_rank` to every rank."""
    if not _ready():
        return obj
    rank = dist.get_rank()
    payload = pickle.dumps(obj) if rank == src_rank else b""
    size = torch.tensor([len(payload)], dtype=torch.long, device=device)
    dist.broadcast(size, src=src_rank)
    buf = torch.zeros(int(size.item()), dtype=torch.uint8, device=device)
    if rank == src_rank and payload:
        buf.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device))
    dist.broadcast(buf, src=src_rank)
    return obj if rank == src_rank else pickle.loads(buf.cpu().numpy().tobytes())


def all_reduce_tensor(tensor: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce; op in {sum, mean, max, min} (mean = sum / world_size)."""
    if not _ready():
        return tensor
    ops = {"sum": dist.ReduceOp.SUM, "mean": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
    if op not in ops:
        raise ValueError(f"Unsupported operation: {op}")
    dist.all_reduce(tensor, op=ops[op])
    if op == "mean":
        tensor /= dist.get_world_size()
    return tensor


def barrier() -> None:
    if _ready():
        dist.barrier()


def replica_checksums(params, device=None):
    """(plain, position-weighted) exact int64 sums of the parameters' fp32 bit patterns, all-reduced
    MAX and MIN over the ranks: data-parallel replicas are bit-identical iff max == min for both (up to
    hash collisions). Returns (identical, local sums, max, min)."""
    ps = [p.detach().reshape(-1) for p in params]
    dev = device or (ps[0].device if ps else "cpu")
    h = torch.zeros(2, dtype=torch.int64, device=dev)
    for i, p in enumerate(ps):
        bits = p.contiguous().view(torch.int32).to(torch.int64)
        h[0] += bits.sum()
        w = (torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 1021) + 1 + i
        h[1] += (bits * w).sum()
    mx, mn = h.clone(), h.clone()
    if _ready():
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    return bool(torch.equal(mx, mn)), h.tolist(), mx.tolist(), mn.tolist()


def broadcast_parameters(tensors, src_rank: int = 0, process_group=None) -> None:
    """Every rank's copies of `tensors` (parameters, buffers) become those of rank src_rank OF
    `process_group` (its group rank; for the default group the global rank), in place: the start
    state data-parallel replicas need, which DistributedDataParallel's constructor sets the same way
    (module states broadcast from the group's rank 0; reference runner.py:703-707). A no-op without
    an initialised process group of more than one rank."""
    if not _ready() or dist.get_world_size(process_group) < 2:
        return
    src = dist.get_global_rank(process_group, src_rank) if process_group is not None else src_rank
    with torch.no_grad():
        for t in tensors:
            dist.broadcast(t.data, src=src, group=process_group)


class GradientSync:
    """Bucketed, backward-overlapped gradient all-reduce over one flat fp32 buffer per bucket.

    usage:  sync = GradientSync(model.parameters())
            loss.backward(); sync.finish(); clip; optimizer.step()

    Buckets follow DDP's reducer (reference runner.py:703-707 wraps the model in DDP with its
    defaults): reverse registration order, a small first bucket (first_bucket_mb, DDP's 1 MiB) so
    the collectives start early in the backward, then bucket_mb (DDP's 25 MiB) buckets.

    `unused`: parameters the model never uses in forward (GNN.long_range_projection, reference
    gnn.py:146): they take no part in the sync and keep grad None, as DDP(find_unused_parameters)
    leaves them; without this their bucket could only start at finish(). Every rank must pass the
    same set.

    Start state: like DDP's constructor, the constructor broadcasts every parameter it is given
    (the unused ones too) from rank 0, so replicas initialised from different seeds start equal
    (`broadcast_params=False` skips it for callers that have synchronised them already).

    Transport: over the "nccl" backend (RCCL) the buckets go through an RCCL communicator of the
    library's own (aimx._lib.Comm, include/aimx.h aimx_comm_*): one ncclAllReduce(ncclAvg) per
    bucket — the average in the collective's own kernel — on a side stream forked from the
    backward's stream by an event and joined back in finish(). torch.distributed's own
    ProcessGroupNCCL is not used for them because its watchdog thread queries every collective's
    event, and events recorded during graph capture may not be queried (the process aborts).
    Over gloo (CPU rehearsal) the buckets use dist.all_reduce.

    Graph capture: with overlap, each bucket's pack + all-reduce is issued from the
    post-accumulate-grad hook of its last gradient; inside torch.cuda.graph capture they become
    graph nodes on the side stream, so a replay runs them concurrently with the rest of the
    backward (aimx.train.GraphedTrainStep "capture" mode). `always=True` runs the bucket path
    even at world size 1 (tests of that mechanism on a one-GPU box).
    """

    def __init__(self, params, bucket_mb: float = 25.0, process_group=None, overlap: bool = True,
                 first_bucket_mb: float = 1.0, unused=(), always: bool = False, broadcast_params: bool = True,
                 auto_finish: bool = False, gate=None, side_stream=None):
        params = list(params)
        unused = list(unused)
        if broadcast_params:
            seen = {id(p) for p in params}
            broadcast_parameters(params + [p for p in unused if id(p) not in seen], 0, process_group)
        skip = {id(p) for p in unused}
        self.params = [p for p in params if p.requires_grad and id(p) not in skip]
        self.group = process_group
        self.world = dist.get_world_size(process_group) if _ready() else 1
        self.active = self.world > 1 or (always and _ready())
        self.overlap = overlap and self.active
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        cap0 = max(1, int(min(first_bucket_mb, bucket_mb) * 1024 * 1024 / 4))
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):  # backward produces late layers first
            limit = cap0 if not self.buckets else cap
            if cur and size + p.numel() > limit:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self._flat = [None] * len(self.buckets)
        self._pending = [0] * len(self.buckets)
        self._handles = [None] * len(self.buckets)
        self._hooks = []
        import os
        # Side stream (overlap with the backward) only for large gradient sets: measured on one
        # MI355X with a world-size-1 RCCL group (profiles/r02_ddp_ab.txt), the forked graph costs
        # ~20 us per c2 step (3.3 MB of gradients: an 8-GPU all-reduce of them is only tens of us)
        # and nothing at c5 (63 MB, where an 8-GPU all-reduce takes ~0.3 ms and overlap pays).
        # side_stream=True / False forces it on / off.
        total = sum(p.numel() for p in self.params) * 4
        self.side_stream = bool(side_stream) if side_stream is not None else total >= 16 * 2 ** 20
        self.comm = None
        self._stream = None
        self._events = []
        if self.active and self.backend == "nccl" and self.params and self.params[0].is_cuda:
            from aimx import _lib
            dev = self.params[0].device
            self.comm = _lib.Comm(process_group, dev)
            self._stream = torch.cuda.Stream(device=dev)
            self._events = [(torch.cuda.Event(), torch.cuda.Event()) for _ in self.buckets]
        # auto_finish: the first bucket hook of a backward queues finish() as an autograd-engine
        # callback (what DDP's reducer does with its finalize), so a loop that never calls finish()
        # — the reference trainer under DistributedDataParallel — still gets averaged gradients
        self.auto_finish = auto_finish
        self._queued = False
        # gate: called at a backward's first gradient; False skips that backward's sync altogether
        # (DistributedDataParallel.no_sync(): the gradients accumulate locally, and the next synced
        # backward's hooks see — and average — the accumulated .grad, as DDP's reducer does)
        self.gate = gate
        if self.overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self.hook_ids = {h.id for h in self._hooks}
        self._reset()

    @property
    def backend(self) -> str:
        return dist.get_backend(self.group) if _ready() else ""

    @property
    def capturable(self) -> bool:
        """True when the collectives can be recorded into a HIP graph (our RCCL communicator;
        gloo runs on the host)."""
        return self.overlap and self.comm is not None

    def _reset(self):
        self._pending = [len(b) for b in self.buckets]
        self._handles = [None] * len(self.buckets)

    def _launch(self, i):
        # one persistent flat buffer per bucket: the gradients are packed by ONE cat kernel into it,
        # all-reduced in place, then scattered back by one multi-tensor copy (finish)
        bucket = self.buckets[i]
        flat = self._flat[i]
        if flat is None or flat.device != bucket[0].device:
            flat = torch.empty(sum(p.numel() for p in bucket), dtype=bucket[0].dtype, device=bucket[0].device)
            self._flat[i] = flat
        if self.comm is not None:
            # pack every gradient (zeros for a missing one) into the flat buffer: one launch
            from aimx import _lib
            pairs, off = [], 0
            for p in bucket:
                n = p.numel()
                g = p.grad
                pairs.append((g if g is not None and g.is_contiguous() else
                              (g.contiguous() if g is not None else None), flat[off:off + n]))
                off += n
            _lib.multi_copy(pairs, flat.device)
        else:
            grads = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in bucket]
            torch.cat(grads, out=flat)
        if self.comm is not None:
            ready, done = self._events[i]
            cur = torch.cuda.current_stream(flat.device)
            side = self._stream if self.side_stream else cur
            if side is not cur:
                ready.record(cur)
                side.wait_event(ready)
            self.comm.all_reduce(flat, average=True, stream=side)
            done.record(side)
            self._handles[i] = done
        else:
            self._handles[i] = dist.all_reduce(flat, group=self.group, async_op=True)

    def new_step(self):
        """Forget a backward that never finished (it raised after its first bucket hook, so the
        engine dropped the queued finish()): called at every training forward of a wrapped model."""
        if self._queued or any(h is not None for h in self._handles):
            self._queued = False
            self._reset()

    def syncing(self):
        """Whether the current backward is synced (the gate, DDP's require_backward_grad_sync)."""
        return self.gate is None or bool(self.gate())

    def _on_grad(self, p):
        if self.auto_finish and not self._queued:
            if not self.syncing():  # a no_sync() backward: every hook of it returns here
                return
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish_queued)
        elif not self.auto_finish and not self.syncing():
            return
        i = self._bucket_of[id(p)]
        self._pending[i] -= 1
        if self._pending[i] == 0 and self._handles[i] is None:
            self._launch(i)

    def _finish_queued(self):
        self._queued = False
        self.finish()

    def reduce_tensors(self, grads, key=None):
        """Average the gradients `grads` ({id(param): tensor}, this sync's parameters) across the
        ranks in place, bucket by bucket on the current stream (pack, one all-reduce, unpack): the
        gradients a graph replay produced without running the parameters' accumulators
        (aimx.autograph). A parameter missing from `grads` counts as zeros. `key` (hashable): the
        same tensors come back every call under it (a replay's static gradients), so the pack /
        unpack launch descriptors are built once (and `grads` holds them alive meanwhile)."""
        if not self.active:
            return
        if key is not None and self.comm is not None:
            cache = self.__dict__.setdefault("_rt_cache", {})
            plan = cache.get(key)
            if plan is None:
                from aimx import _lib
                plan = []
                for i, bucket in enumerate(self.buckets):
                    flat = self._flat[i]
                    if flat is None or flat.device != bucket[0].device:
                        flat = torch.empty(sum(p.numel() for p in bucket), dtype=bucket[0].dtype,
                                           device=bucket[0].device)
                        self._flat[i] = flat
                    pairs, back, off = [], [], 0
                    for p in bucket:
                        n = p.numel()
                        g = grads.get(id(p))
                        pairs.append((g.reshape(-1) if g is not None else None, flat[off:off + n]))
                        if g is not None:
                            back.append((flat[off:off + n], g.reshape(-1)))
                        off += n
                    plan.append((flat, _lib.copy_items(pairs), _lib.copy_items(back), pairs, back))
                if len(cache) > 8:
                    cache.clear()
                cache[key] = plan
            from aimx import _lib
            for flat, pack, unpack, _, _ in plan:
                _lib.multi_copy_items(pack, flat.device)
                self.comm.all_reduce(flat, average=True, stream=torch.cuda.current_stream(flat.device))
                _lib.multi_copy_items(unpack, flat.device)
            return
        for i, bucket in enumerate(self.buckets):
            flat = self._flat[i]
            if flat is None or flat.device != bucket[0].device:
                flat = torch.empty(sum(p.numel() for p in bucket), dtype=bucket[0].dtype, device=bucket[0].device)
                self._flat[i] = flat
            pairs, back, off = [], [], 0
            for p in bucket:
                n = p.numel()
                g = grads.get(id(p))
                pairs.append((g.reshape(-1) if g is not None else None, flat[off:off + n]))
                if g is not None:
                    back.append((flat[off:off + n], g.reshape(-1)))
                off += n
            if self.comm is not None:
                from aimx import _lib
                _lib.multi_copy(pairs, flat.device)
                self.comm.all_reduce(flat, average=True, stream=torch.cuda.current_stream(flat.device))
                if back:
                    _lib.multi_copy(back, flat.device)
            else:
                torch.cat([g if g is not None else torch.zeros_like(d) for g, d in pairs], out=flat)
                dist.all_reduce(flat, group=self.group)
                if self.world > 1:
                    flat.div_(self.world)
                if back:
                    torch._foreach_copy_([d for _, d in back], [s_ for s_, _ in back])

    def finish(self):
        """Complete every bucket's all-reduce and write averaged gradients back into .grad."""
        if not self.active or not self.syncing():
            self._reset()
            return
        for i in range(len(self.buckets)):
            if self._handles[i] is None:
                self._launch(i)
        for i, bucket in enumerate(self.buckets):
            flat = self._flat[i]
            if self.comm is not None:  # averaged by the collective (ncclAvg); join its stream
                torch.cuda.current_stream(flat.device).wait_event(self._handles[i])
            else:
                self._handles[i].wait()
                if self.world > 1:
                    flat.div_(self.world)
            dst, src, off = [], [], 0
            for p in bucket:
                n = p.numel()
                if p.grad is not None:
                    dst.append(p.grad)
                    src.append(flat[off:off + n].view_as(p))
                off += n
            if dst and self.comm is not None and all(d.is_contiguous() for d in dst):
                from aimx import _lib
                _lib.multi_copy(list(zip(src, dst)), flat.device)  # one launch for the bucket
            elif dst:
                torch._foreach_copy_(dst, src)
        self._reset()

    def time_allreduce(self, iters: int = 20) -> float:
        """Microseconds per step of this sync's collectives alone: every bucket's all-reduce on its
        flat buffer, back to back, `iters` times (HIP events on the collectives' stream for RCCL,
        wall clock for gloo). Call after training steps (the flat buffers exist; their contents
        are scratch until the next pack)."""
        import time
        if not self.active or any(f is None for f in self._flat):
            return 0.0
        dev = self._flat[0].device
        if self.comm is not None:
            s = self._stream if self.side_stream else torch.cuda.current_stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for f in self._flat:  # warm
                self.comm.all_reduce(f, average=True, stream=s)
            t0.record(s)
            for _ in range(iters):
                for f in self._flat:
                    self.comm.all_reduce(f, average=True, stream=s)
            t1.record(s)
            t1.synchronize()
            torch.cuda.current_stream(dev).wait_stream(s)
            return t0.elapsed_time(t1) * 1e3 / iters
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(iters):
            for f in self._flat:
                dist.all_reduce(f, group=self.group)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) * 1e6 / iters

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self.comm is not None:
            self.comm.close()
            self.comm = None
