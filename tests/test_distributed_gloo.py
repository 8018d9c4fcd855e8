"""Multi-process (world_size 2, gloo, CPU) tests of utils/distributed.py: the reference helper API
(rank-0 return conventions) and GradientSync's DDP-equivalent averaging, with and without the
backward-overlapped bucket hooks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn_name, q):
    import sys
    sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, globals()[fn_name](rank, world)))
    finally:
        dist.destroy_process_group()


def _run(fn_name, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=120)
        out[r] = v
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _helpers(rank, world):
    from utils import distributed as D
    arr = np.arange(3 + rank, dtype=np.float32).reshape(-1, 1) + 10 * rank
    g = D.gather_ndarray_to_rank0(arr)
    s = D.gather_strings_to_rank0([f"r{rank}a", f"r{rank}b"])
    b = D.broadcast_object({"best": 1.5, "stop": rank == 0} if rank == 0 else None)
    t = D.all_reduce_tensor(torch.tensor([float(rank + 1)]), "mean")
    m = D.all_reduce_tensor(torch.tensor([float(rank + 1)]), "max")
    D.barrier()
    return dict(g=g.tolist(), s=s, b=b, t=t.item(), m=m.item(), rank=D.safe_get_rank(), ws=D.get_world_size(),
                main=D.is_main_process())


def test_reference_helpers():
    out = _run("_helpers")
    assert out[0]["g"] == [[0.0], [1.0], [2.0], [10.0], [11.0], [12.0], [13.0]] and out[1]["g"] == []
    assert out[0]["s"] == ["r0a", "r0b", "r1a", "r1b"] and out[1]["s"] == []
    assert out[0]["b"] == out[1]["b"] == {"best": 1.5, "stop": True}
    assert out[0]["t"] == out[1]["t"] == 1.5 and out[0]["m"] == 2.0
    assert out[0]["main"] and not out[1]["main"] and out[1]["rank"] == 1 and out[0]["ws"] == 2


def _grad_sync(rank, world):
    from utils.distributed import GradientSync
    res = {}
    for overlap in (True, False):
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.SiLU(), torch.nn.Linear(5, 3),
                                  torch.nn.Linear(3, 3))  # last layer unused below -> grad None
        sync = GradientSync(net.parameters(), bucket_mb=0.0001, overlap=overlap)
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(4, 7, generator=g)
        net[2](net[1](net[0](x))).pow(2).sum().backward()
        sync.finish()
        res[overlap] = {n: (p.grad.clone().tolist() if p.grad is not None else None)
                        for n, p in net.named_parameters()}
        sync.remove()
    return res


def test_gradient_sync_equals_mean_of_rank_gradients():
    out = _run("_grad_sync")
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.SiLU(), torch.nn.Linear(5, 3), torch.nn.Linear(3, 3))
    grads = []
    for rank in range(2):
        net.zero_grad()
        x = torch.randn(4, 7, generator=torch.Generator().manual_seed(100 + rank))
        net[2](net[1](net[0](x))).pow(2).sum().backward()
        grads.append({n: (p.grad.clone() if p.grad is not None else None) for n, p in net.named_parameters()})
    for overlap in (True, False):
        for n, _ in net.named_parameters():
            if grads[0][n] is None:
                assert out[0][overlap][n] is None and out[1][overlap][n] is None
                continue
            want = (grads[0][n] + grads[1][n]) / 2
            for r in range(2):
                assert torch.allclose(torch.tensor(out[r][overlap][n]), want, atol=1e-6), (n, overlap)


def test_gradient_sync_bucket_layout():
    """DDP's reducer layout: reverse registration order, a small first bucket, unused params out."""
    from utils.distributed import GradientSync
    net = torch.nn.Sequential(torch.nn.Linear(512, 512), torch.nn.Linear(512, 512), torch.nn.Linear(512, 512),
                              torch.nn.Linear(512, 4))
    sync = GradientSync(net.parameters(), bucket_mb=2.0, first_bucket_mb=1.0, unused=list(net[1].parameters()))
    names = {id(p): n for n, p in net.named_parameters()}
    layout = [[names[id(p)] for p in b] for b in sync.buckets]
    assert layout[0] == ["3.bias", "3.weight", "2.bias"]  # 2.weight (1 MiB) would overflow the 1 MiB first bucket
    assert all("1." not in n for b in layout for n in b)
    assert sum(len(b) for b in layout) == 6
    for b in sync.buckets[1:]:
        assert sum(p.numel() for p in b) * 4 <= 2 * 2 ** 20 or len(b) == 1
    assert not sync.active and not sync.capturable  # no process group: finish() is a no-op
    sync.finish()


def _checksums(rank, world):
    from utils.distributed import GradientSync, replica_checksums
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
    same = replica_checksums(list(net.parameters()))[0]
    with torch.no_grad():
        if rank == 1:  # one ulp on one replica
            w = net[0].weight.view(-1)
            w[3] = torch.nextafter(w[3], torch.tensor(float("inf")))
    differ = replica_checksums(list(net.parameters()))[0]
    sync = GradientSync(net.parameters(), bucket_mb=0.0001)
    net(torch.randn(2, 7)).sum().backward()
    sync.finish()
    us = sync.time_allreduce(iters=3)
    return {"same": same, "differ": differ, "us": us, "buckets": len(sync.buckets)}


def test_replica_checksums_and_allreduce_timing():
    """bench.py's self-check of a data-parallel run: identical replicas agree, one ulp of difference
    on one rank is caught on every rank; the collectives' own time per step is measured."""
    out = _run("_checksums")
    for r in range(2):
        assert out[r]["same"] and not out[r]["differ"], out[r]
        assert out[r]["us"] > 0 and out[r]["buckets"] >= 2


def _start_state(rank, world):
    """Replicas built from different seeds (bench.py seeds per rank): GradientSync's constructor
    broadcasts rank 0's parameters (DDP's constructor does the same), the unused ones included, so
    after identical averaged steps every replica is bit-identical (replica_checksums)."""
    from utils.distributed import GradientSync, replica_checksums
    torch.manual_seed(100 + rank)
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.SiLU(), torch.nn.Linear(5, 3), torch.nn.Linear(3, 3))
    before = replica_checksums(net.parameters())[0]
    sync = GradientSync(net.parameters(), bucket_mb=0.0001, unused=list(net[3].parameters()))
    after = replica_checksums(net.parameters())[0]
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(rank)
    for _ in range(3):
        opt.zero_grad()
        net[:3](torch.randn(4, 7, generator=g)).pow(2).sum().backward()
        sync.finish()
        opt.step()
    return before, after, replica_checksums(net.parameters())[0]


def test_gradient_sync_broadcasts_start_state():
    out = _run("_start_state")
    for r in (0, 1):
        before, after, trained = out[r]
        assert not before and after and trained


def _subgroup_broadcast(rank, world):
    """broadcast_parameters over a subgroup that does not hold global rank 0: the source is the
    GROUP's rank 0 (global rank 1), as DDP's constructor does."""
    from utils.distributed import broadcast_parameters
    grp = dist.new_group([1, 2])
    t = torch.full((4,), float(rank))
    if rank in (1, 2):
        broadcast_parameters([t], 0, grp)
    dist.barrier()
    return t.tolist()


def test_broadcast_parameters_subgroup_source():
    out = _run("_subgroup_broadcast", world=3)
    assert out[0] == [0.0] * 4
    assert out[1] == [1.0] * 4 and out[2] == [1.0] * 4


def _ddp_wrap_native(rank, world):
    """The reference's wrap, unchanged (runner.py:703-707), around the GNN on CPU (construction only:
    the forward needs the GPU): DDP reads GNN._ddp_params_and_buffers_to_ignore, keeps the anchor
    parameter alone in its reducer, and the model broadcasts its own start state."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    from models import GNN
    from utils.distributed import replica_checksums
    torch.manual_seed(100 + rank)  # different start states on the two ranks
    m = GNN({"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}, 64, 1)
    before = replica_checksums(m.parameters())[0]
    ddp = DDP(m, find_unused_parameters=True)
    kept = [n for n, _ in m.named_parameters() if n not in ddp.parameters_to_ignore]
    after = replica_checksums(m.parameters())[0]
    native = m.__dict__.get("_aimx_ddp_native", False)
    os.environ["AIMX_NATIVE_DDP"] = "0"
    m2 = GNN({"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}, 64, 1)
    ddp2 = DDP(m2, find_unused_parameters=True)
    plain_ignored = len(ddp2.parameters_to_ignore)
    del os.environ["AIMX_NATIVE_DDP"]
    return before, after, kept, native, plain_ignored, len(list(m.named_parameters()))


def test_ddp_wrap_keeps_one_parameter_and_syncs_start_state():
    out = _run("_ddp_wrap_native")
    for r in (0, 1):
        before, after, kept, native, plain_ignored, n = out[r]
        assert not before and after  # rank 0's parameters everywhere after the wrap
        assert kept == ["output_layer.bias"] and native and n == 73
        assert plain_ignored == 0  # AIMX_NATIVE_DDP=0: DDP keeps every parameter


def _fake_backward(params, scale):
    """A backward whose gradient of every parameter is `scale` (ones · scale): fires the sync's
    post-accumulate-grad hooks exactly as a model backward does."""
    loss = sum((p * scale).sum() for p in params)
    loss.backward()


def _ddp_subgroup_and_no_sync(rank, world):
    """DDP(model, process_group=subgroup) on ranks 1 and 2 of 3: the native sync follows the
    wrapper's group (start state from the GROUP's rank 0, gradients averaged over the group only),
    and ddp.no_sync() micro-batches accumulate locally; the next synced backward averages the
    accumulated gradients (DDP's semantics)."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    from models import GNN
    grp = dist.new_group([1, 2])
    if rank not in (1, 2):
        dist.barrier()
        return None
    torch.manual_seed(100 + rank)
    m = GNN({"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}, 64, 1)
    ddp = DDP(m, process_group=grp, find_unused_parameters=True)
    sync = m._aimx_native_sync()
    assert sync.group is grp and sync.world == 2
    params = sync.params
    # two no_sync micro-batches (local scale rank, then 2*rank), then one synced (3*rank)
    with ddp.no_sync():
        sync.new_step()
        _fake_backward(params, float(rank))
        sync.new_step()
        _fake_backward(params, 2.0 * rank)
    local = params[0].grad.flatten()[0].item()
    sync.new_step()
    _fake_backward(params, 3.0 * rank)
    synced = params[0].grad.flatten()[0].item()
    try:  # uneven inputs (DDP.join) are refused with a clear error, not silently mis-synced
        with ddp.join():
            m._aimx_native_sync()
        joined = "no error"
    except Exception as e:
        joined = type(e).__name__
    dist.barrier()
    return local, synced, joined, [p.detach().flatten()[:8].tolist() for p in list(m.parameters())[:2]]


def test_ddp_native_sync_follows_group_and_no_sync():
    out = _run("_ddp_subgroup_and_no_sync", world=3)
    assert out[0] is None
    l1, s1, j1, p1 = out[1]
    l2, s2, j2, p2 = out[2]
    assert j1 == j2 == "AimxError"
    assert l1 == 3.0 and l2 == 6.0                 # no_sync: local sums only (1+2, 2+4)
    assert s1 == s2 == (6.0 + 12.0) / 2            # synced: the accumulated sums averaged over {1, 2}
    assert p1 == p2  # start state from the group's rank 0


def test_param_key_sees_storage_swaps():
    """autograph re-captures when a parameter's storage moves without any registration
    (`p.data = ...`: torch.nn.utils.vector_to_parameters, EMA / SWA swaps)."""
    from aimx import autograph
    from models import GNN
    m = GNN({"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}, 64, 1)
    k0 = autograph._param_key(m)
    assert autograph._param_key(m) == k0
    p = next(m.parameters())
    p.data = p.data.clone()
    assert autograph._param_key(m) != k0
