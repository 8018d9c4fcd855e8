"""Throughput bench of the AIMNet-X2D hot path on MI355X (BASELINE.json metric).

metric: molecules/sec of a full training step (forward + backward + grad-norm clip 1.0 + Adam,
dropout on, L1 loss) on QM9-shaped batches, plus the achieved HBM GB/s of the scatter-add hop.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
  N > 1: `python bench.py --gpus N` starts its own N rank processes (launch_ranks, one GPU each);
         under torchrun (`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`)
         it uses the launcher's ranks. --gpus must equal WORLD_SIZE, or the command fails.

Workload (default c2 = BASELINE configs[1]): QM9, hidden 256, 3 hops, 512 molecules per GPU per
step, single task, attention pooling. Data: synthetic QM9-shaped batches resampled from the
committed QM9-val graph asset (rng 1234 + rank), collated by aimx.data and resident in HBM
before timing; weights random (GNN.init_weights). Each rank trains on its own molecules (weak
scaling); gradients are averaged with one bucketed RCCL all-reduce per step (GradientSync).
Rank 0 prints one JSON line. `roofline` times the hop kernel alone at the roofline size
(4M QM9-shaped atoms, working set >> 256 MiB MALL) with HIP events on its launch stream;
`cpu_baseline` times the oracle's CPU restatement of the reference train step (kind "port") on a
bounded sample at N = 1.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aimnet-x2d_amd")]

from aimx import data as adata  # noqa: E402
from aimx import ops  # noqa: E402
from aimx.synth import QM9Asset, synth_molecules  # noqa: E402

CONFIGS = {
    "c1": dict(source="qm9", hidden=128, hops=3, batch=32, tasks=1, pc=False),
    "c2": dict(source="qm9", hidden=256, hops=3, batch=512, tasks=1, pc=False),
    "c3": dict(source="qm9", hidden=256, hops=4, batch=512, tasks=12, pc=True),
    "c4": dict(source="synth40", hidden=512, hops=3, batch=512, tasks=1, pc=False, quantum=32),
    "c5": dict(source="synth40", hidden=1024, hops=6, batch=256, tasks=1, pc=False, quantum=32),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FS = {"atom_type": 119, "hydrogen_count": 9, "degree": 7, "hybridization": 7}


def make_collated(cfg, n_batches, seed):
    """Host-collated batches (aimx.data) with targets and total charges."""
    rng = np.random.default_rng(seed)
    out = []
    if cfg["source"] == "qm9":
        asset = QM9Asset()
        for _ in range(n_batches):
            idx = rng.integers(0, len(asset), cfg["batch"])
            col = adata.collate(asset.molecules(idx), cfg["hops"])
            tg = asset.targets[idx][:, : cfg["tasks"]].astype(np.float32)
            tg = (tg - tg.mean(0)) / (tg.std(0) + 1e-6)
            out.append((col, tg, asset.total_charge[idx].astype(np.float32)))
    else:
        for _ in range(n_batches):
            mols = synth_molecules(cfg["batch"], seed=int(rng.integers(1 << 30)))
            col = adata.collate(mols, cfg["hops"])
            tg = rng.standard_normal((cfg["batch"], cfg["tasks"])).astype(np.float32)
            out.append((col, tg, np.zeros(cfg["batch"], np.float32)))
    return out


PAD_MOLS = 8  # padding molecules appended to each static batch (excluded from the loss)
# atoms: one-GPU static batches are padded to the next multiple (one graph each). c4 / c5 (device-
# bound steps, no launch overhead for the graph to win back) use 32: every padded atom is paid in
# full there (profiles/r05_quantum_ab.txt: c5 graphed 3.972 -> 3.952 ms, eager 3.965-3.975; c4
# 2.600 -> 2.590); c2 keeps 128 (0.7249 vs 0.7324 ms with 32). --quantum overrides (A/B).
LAYOUT_QUANTUM = 128
QUANTUM_OVERRIDE = None


def layout_quantum(cfg):
    return int(QUANTUM_OVERRIDE or cfg.get("quantum", LAYOUT_QUANTUM))


def make_batches(cfg, n_batches, seed, device, pad=False, buckets=False):
    """Device-resident batches. pad=True: static shapes for graph replay (padding molecules of at
    most 64 atoms each, pad_mols_for) — one shape for all (max atoms + 64, max edges + 256, at least
    PAD_MOLS padding molecules), or with `buckets` one per atom-count bucket (real atoms + 2 rounded up
    to LAYOUT_QUANTUM, the bucket's max edges + 64, as few padding molecules as keep each within 64
    atoms), each captured as its own graph by GraphedTrainStep."""
    cols = make_collated(cfg, n_batches, seed)
    if not pad:
        return [adata.DeviceBatch(c, device, targets=t, total_charges=q, csr_hops=cfg["hops"]) for c, t, q in cols]

    q = layout_quantum(cfg)

    def bucket(c):
        n = c["batch"].shape[0]
        return -(-(n + 2) // q) * q if buckets else 0
    groups = {}
    for c, _, _ in cols:
        groups.setdefault(bucket(c), []).append(c)
    shape = {}
    for k, cs in groups.items():
        n_max = k or max(c["batch"].shape[0] for c in cs) + 64
        n_min = min(c["batch"].shape[0] for c in cs)
        e_max = max(c["edges"].shape[0] for c in cs) + (64 if k else 256)
        shape[k] = (n_max, e_max, adata.pad_mols_for(n_max, n_min, 64, 1) if k else pad_mols_for(n_max, n_min))
    out = []
    for c, t, chg in cols:
        n_max, e_max, pm = shape[bucket(c)]
        real_atoms, real_edges = c["batch"].shape[0], c["edges"].shape[0]
        pc = adata.pad_collated(c, n_max, e_max, cfg["batch"], pm)
        tg = np.concatenate([t, np.zeros((pm, t.shape[1]), np.float32)])
        qq = np.concatenate([chg, np.zeros(pm, np.float32)])
        b = adata.DeviceBatch(pc, device, targets=tg, total_charges=qq, csr_hops=cfg["hops"])
        b.real_atoms, b.real_edges, b.real_graphs = real_atoms, real_edges, cfg["batch"]
        out.append(b)
    return out


def native_feeder(cfg, seed, device, threads, pad):
    """Endless BatchFeeder over a molecule store (C++ batch builder, aimx/feed.py): random batches
    of cfg['batch'] molecules, padded to static shapes for graph replay when `pad`."""
    from aimx import feed
    rng = np.random.default_rng(seed)
    if cfg["source"] == "qm9":
        asset = QM9Asset()
        store = feed.HostStore.from_arrays(asset.atom_off, asset.bond_off, np.stack([asset.bi, asset.bj], 1),
                                           asset.feats, asset.targets[:, : cfg["tasks"]], asset.total_charge,
                                           precompute_hops=cfg["hops"], threads=threads)
    else:
        mols = synth_molecules(8192, seed=seed)
        store = feed.HostStore.from_molecules(mols, rng.standard_normal((len(mols), cfg["tasks"])),
                                              precompute_hops=cfg["hops"], threads=threads)
    B = cfg["batch"]
    n_max = e_max = pm = 0
    if pad:  # static capacity from 256 sampled batches (a batch over it is stepped eagerly)
        n_max, e_max, pm = feed.static_capacity(feed.HostCollator(cfg["hops"], threads), store,
                                                [rng.integers(0, len(store), B) for _ in range(256)],
                                                least_pad_mols=PAD_MOLS)

    def index_stream():
        while True:
            yield rng.integers(0, len(store), B)
    # ring: GraphedTrainStep copies every batch into its static inputs before asking for the next
    return iter(feed.BatchFeeder(store, index_stream(), cfg["hops"], device, depth=4, threads=threads,
                                 n_max=n_max, e_max=e_max, pad_mols=pm, ring=pad))


def pad_mols_for(n_max, n_min):
    """Padding molecules of at most 64 atoms each (aimx.data.pad_mols_for; at least PAD_MOLS)."""
    return adata.pad_mols_for(n_max, n_min, 64, PAD_MOLS)


STREAM_INFO = {}


def stream_feeder(cfg, rank, world, device, threads, pad, n_mols, path=None, read_threads=None):
    """Endless BatchFeeder over an HDF5 molecule stream in the reference's dataset format
    (features.py:381-431 / molecular.py:102-329): a synthetic file of n_mols molecules (made once
    on this host by rank 0), this rank's equal shard read in chunks by the C++ reader (HDF5 C
    library + non-executing record decoder) on a prefetch thread, collated by the C++ batch
    builder and copied host->device by BatchFeeder (aimx/h5.py, aimx/feed.py)."""
    from aimx import feed, h5
    path = path or os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                f"aimx_stream_{cfg['source']}_{cfg['hops']}h_{cfg['tasks']}t_{n_mols}.h5")
    info = {"path": path, "molecules": n_mols}
    if rank == 0 and not os.path.exists(path):
        t0 = time.perf_counter()
        tmp = path + f".part{os.getpid()}"
        h5.make_synthetic_stream(tmp, n_mols, cfg["source"], cfg["hops"], cfg["tasks"], seed=0,
                                 workers=min(16, os.cpu_count() or 4))
        os.replace(tmp, path)
        info["write_s"] = round(time.perf_counter() - t0, 1)
        print(f"bench: wrote {n_mols}-molecule stream {path} in {info['write_s']} s", file=sys.stderr)
    if world > 1:
        dist.barrier()
    read_threads = read_threads or threads
    stream = h5.HDF5MolecularStream(path, shuffle=True, ddp_enabled=world > 1, rank=rank, world_size=world,
                                    n_hops=cfg["hops"], n_tasks=cfg["tasks"], threads=read_threads)
    # the reader's own rate (shuffled positions, the feed's threads): read + decode + pack into stores
    pos = stream.positions(0)[:65536]
    t0 = time.perf_counter()
    for s0 in range(0, len(pos), 16384):
        stream.file.read_store(pos[s0:s0 + 16384], cfg["hops"], cfg["tasks"], read_threads)
    info.update(bytes=os.path.getsize(path), direct_read=stream.file.direct_read,
                read_mol_per_s=round(len(pos) / (time.perf_counter() - t0)), read_threads=read_threads)
    STREAM_INFO.update(info)
    B = cfg["batch"]
    n_max = e_max = pm = 0
    if pad:  # static capacity from 256 batches of the first chunk (a batch over it is stepped eagerly)
        store, _ = stream.file.read_store(stream.positions(0)[:16384], cfg["hops"], cfg["tasks"], threads)
        rng = np.random.default_rng(rank)
        n_max, e_max, pm = feed.static_capacity(feed.HostCollator(cfg["hops"], threads), store,
                                                [rng.integers(0, len(store), B) for _ in range(256)],
                                                least_pad_mols=PAD_MOLS)

    def batches():
        epoch = 0
        while True:
            yield from stream.batches(B, chunk_size=16384, epoch_seed=epoch)
            epoch += 1
    return iter(feed.BatchFeeder(None, batches(), cfg["hops"], device, depth=4, threads=threads,
                                 n_max=n_max, e_max=e_max, pad_mols=pm, ring=pad))


def build_model(cfg, device):
    from models import GNN
    m = GNN(FS, cfg["hidden"], cfg["tasks"], num_shells=cfg["hops"], use_partial_charges=cfg["pc"])
    return m.to(device).train()


def hop_kernel(d):
    """The hop kernel that runs for width d: hop.hip for 16-byte rows, else hop_unal.hip."""
    return "k_gather_sum" if d % 4 == 0 else "k_gather_unal"


def hop_roofline(batch, hops, device, hidden=256, target_atoms=4_000_000, launches=20):
    """Time the hop kernel alone on a QM9-shaped graph of ~target_atoms atoms (tiled copies of a
    real collated batch), with HIP events on the stream it is launched on."""
    from aimx import ops
    from aimx.plan import GraphPlan
    n0 = batch.num_atoms
    d = int(0.3 * hidden)
    # the hop kernel indexes its output with 32-bit thread ids (rows * D < 2^31, hop.hip): wide
    # configs (c5: 6 hops x 307 columns) get a proportionally smaller probe graph
    target_atoms = min(target_atoms, int(0.95 * (2 ** 31 - 1) / (hops * d)))
    reps = max(1, target_atoms // n0)
    e0 = batch.edges
    off = (torch.arange(reps, device=device, dtype=torch.int64) * n0).view(reps, 1, 1)
    edges = (e0.unsqueeze(0) + off).reshape(-1, 2)
    n = n0 * reps
    e = edges.shape[0]
    # molecule ids of the tiled graph: the model's plans always carry them (segment-aligned tiles)
    g0 = batch.num_graphs
    mol = (batch.batch.unsqueeze(0) + torch.arange(reps, device=device, dtype=torch.int64).view(reps, 1) * g0)
    plan = GraphPlan(n, hops, edges=edges, batch=mol.reshape(-1), num_graphs=g0 * reps)
    x = torch.randn(n, d, device=device)
    del edges
    torch.cuda.synchronize()
    for _ in range(3):
        ops.hop(plan, x)
    stream = torch.cuda.current_stream()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(stream)
    for _ in range(launches):
        ops.hop(plan, x)
    t1.record(stream)
    t1.synchronize()
    ms = t0.elapsed_time(t1) / launches
    alg_bytes = 4 * (n * d + e + (hops * n + 1) + hops * n * d)
    gbs = alg_bytes / (ms * 1e-3) / 1e9
    traffic = bwd_traffic = None
    tname = "hop_traffic.json" if d % 4 == 0 else f"hop_traffic_d{d}.json"
    tp = os.path.join(ROOT, "profiles", tname)
    if os.path.exists(tp):
        try:
            rec = json.load(open(tp))
            if rec.get("atoms") == n and rec.get("edges") == e and rec.get("kernel", hop_kernel(d)) == hop_kernel(d):
                traffic = rec.get("hbm_bytes_per_launch")
                bwd_traffic = (rec.get("bwd") or {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    bwd = hop_bwd_roofline(plan, n, d, hops, device)
    bwd["traffic"] = bwd_traffic
    del plan, x
    torch.cuda.empty_cache()
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": (f"profiles/{tname}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same "
                               "command (bench.py --roofline-only), per launch, gfx950 corrections applied; not "
                               "measured inside this run") if traffic is not None else None,
            "bwd": bwd,
            "kernel": hop_kernel(d) + " (hop fwd)", "atoms": n, "edges": e,
            "D": d, "hops": hops,
            "algorithmic_bytes_per_launch": alg_bytes, "ms_per_launch": round(ms, 4)}


def graph_time_us(fn, launches=20, replays=5):
    """Device time per launch of fn(): `launches` back-to-back launches captured in one HIP graph on
    a side stream, replayed `replays` times between HIP events recorded on that same stream (eager
    Python launches of a ~10 us kernel would time the host instead). Includes the ~1.5 us boundary
    between dependent kernels."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(launches):
            fn()
    with torch.cuda.stream(s):
        g.replay()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(s)
        for _ in range(replays):
            g.replay()
        t1.record(s)
    t1.synchronize()
    us = t0.elapsed_time(t1) / (replays * launches) * 1e3
    del g
    return us


def _bw(name, bytes_, us, **kw):
    gbs = bytes_ / (us * 1e-6) / 1e9
    return {"kernel": name, "bound": "hbm", "algorithmic_bytes": int(bytes_), "us_per_launch": round(us, 2),
            "achieved": round(gbs, 1), "unit": "GB/s", "peak": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4), **kw}


def cold_time_us(fn, device, launches=20, flush_mb=512):
    """Device time per launch of fn() with a cold MALL / L2: each launch is bracketed by HIP
    events on the current stream right behind a `flush_mb` zero fill (larger than the 256 MiB
    Infinity Cache), which also keeps the GPU busy while the host enqueues the bracketed launch,
    so the events see no launch gap. The mean over `launches`."""
    flush = torch.empty(flush_mb * 2 ** 20 // 4, device=device)
    stream = torch.cuda.current_stream(device)
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    for e0, e1 in ev:
        flush.zero_()
        e0.record(stream)
        fn()
        e1.record(stream)
    torch.cuda.synchronize()
    us = sum(e0.elapsed_time(e1) for e0, e1 in ev) / launches * 1e3
    del flush
    return us


def hop_in_step(batch, hops, hidden, device):
    """The hop forward and backward exactly as one train step's stack runs them per layer
    (stack.hip), at the config's own batch, through the C ABI, cold MALL (cold_time_us):
      forward : src F[:, :D] (row stride LF = K = D (h+1) rounded up to 4 floats, as
                aimx.ops._stack_strides lays the stack out), output written into F's columns
                [D, K) (hop chunk j at column offset D + j D);
      backward: the gathered rows dF[:, D:] at the targets (every target is < N for reference
                inputs, layers.py:154, so chunk 0 only), plus the chunk-0 gradient dF[:, :D] and
                the outer residual dY (row stride LA = D rounded up to 4) added, written into the
                next-lower layer's dY buffer (row stride LA).
    Algorithmic bytes: fwd 4 [N D + E + (h N + 1) + w N D], w = the chunks the step writes (the
    stack skips the trailing edge-less ones, which its GEMMs trim: chunk 0 only for reference inputs);
    bwd 4 [N D (gathered rows) + E + (N + 1) + 2 N D (the residual reads) + N D (written)]."""
    from aimx import _lib
    from aimx.plan import GraphPlan
    lib = _lib.load()
    P = _lib.ptr
    from aimx import ops
    n, d = batch.num_atoms, int(0.3 * hidden)
    K = d * (hops + 1)
    LF, _, LA = ops._stack_strides(d, K)
    plan = GraphPlan(n, hops, edges=batch.edges, batch=batch.batch, num_graphs=batch.num_graphs)
    e = plan.E
    F = torch.randn(n, LF, device=device)
    dF = torch.randn(n, LF, device=device)
    dY = torch.randn(n, LA, device=device)    # the layer's upstream gradient (the outer residual)
    nxt = torch.empty(n, LA, device=device)  # the next-lower layer's dY buffer
    seg, seg_st = plan.row_seg()
    s = _lib.stream_ptr(device)
    fl = 4  # bytes per float: column offsets as pointer arithmetic
    kern = hop_kernel(d)

    def fwd():  # the stack's call: trailing edge-less chunks not written (AIMX_GATHER_SKIP_TAIL)
        assert lib.aimx_segment_gather_sum_ex(P(F), LF, 0, 0, d, P(plan.fwd.rowptr), P(plan.fwd.col), hops * n,
                                              P(F) + fl * d, LF, n, d, None, 0, None, 0, seg, seg_st,
                                              _lib.GATHER_SKIP_TAIL, s) == 0

    def bwd():
        assert lib.aimx_segment_gather_sum(P(dF) + fl * d, LF, n, d, d, P(plan.bwd.rowptr), P(plan.bwd.col), n,
                                           P(nxt), LA, 0, 0, P(dF), LF, P(dY), LA, seg, seg_st, s) == 0
    # chunks the step writes: up to the last one holding an edge (reference inputs: chunk 0 only)
    rp = plan.fwd.rowptr.cpu()
    written = max([k + 1 for k in range(hops) if int(rp[(k + 1) * n]) > int(rp[k * n])], default=0)
    torch.cuda.synchronize()
    tf, tb = cold_time_us(fwd, device), cold_time_us(bwd, device)
    bf = 4 * (n * d + e + (hops * n + 1) + written * n * d)
    bb = 4 * (n * d + e + (n + 1) + 2 * n * d + n * d)
    note = (f"the stack's own layout (F row stride {LF}, chunk column offset D; dY / output row stride {LA}; "
            "residual adds), cold MALL (512 MiB flush per launch)")
    return {"atoms": n, "edges": e, "D": d, "hops": hops, "chunks_written": written,
            "fwd": _bw(kern + " (hop fwd, in-step layout)", bf, tf, timing=note),
            "bwd": _bw(kern + " (hop bwd + residual adds, in-step layout)", bb, tb, timing=note)}


def hop_bwd_roofline(plan, n, d, hops, device, launches=20):
    """Hop backward at the roofline size (HIP events on the launch stream, like hop_roofline)."""
    from aimx import _lib
    lib = _lib.load()
    P = _lib.ptr
    g = torch.randn(hops * n, d, device=device)
    dx = torch.empty(n, d, device=device)
    seg, seg_st = plan.row_seg()
    s = _lib.stream_ptr(device)

    def bwd():
        assert lib.aimx_segment_gather_sum(P(g), d, 0, 0, d, P(plan.bwd.rowptr), P(plan.bwd.col), n, P(dx), d, 0, 0,
                                           None, 0, None, 0, seg, seg_st, s) == 0
    for _ in range(3):
        bwd()
    stream = torch.cuda.current_stream()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(stream)
    for _ in range(launches):
        bwd()
    t1.record(stream)
    t1.synchronize()
    us = t0.elapsed_time(t1) / launches * 1e3
    # bytes: the gathered rows (chunk 0 only for reference inputs) + col + rowptr + dx written
    return _bw(hop_kernel(d) + " (hop bwd)",
               4 * (n * d + plan.E + (n + 1) + n * d), us)


def attn_in_step(batch, hidden, device, heads=4):
    """Attention pool forward/backward (pool.hip) at the config's batch, through the C ABI.
    Algorithmic bytes (fp32): fwd = read x, W; write attn, scores, pooled; bwd = read x, attn,
    scores, dpooled, W; write dx, dW."""
    from aimx import _lib
    from aimx.plan import GraphPlan
    lib = _lib.load()
    P = _lib.ptr
    n, C, G, H = batch.num_atoms, hidden, batch.num_graphs, heads
    plan = GraphPlan(n, 1, batch=batch.batch, num_graphs=G)
    x = torch.randn(n, C, device=device)
    W, b = torch.randn(H, C, device=device) * C ** -0.5, torch.zeros(H, device=device)
    tau = torch.ones(1, device=device)
    pooled, attn, scores = (torch.empty(G, C, device=device), torch.empty(H, n, device=device),
                            torch.empty(H, n, device=device))
    dpool, dx = torch.randn(G, C, device=device), torch.empty(n, C, device=device)
    dW, db, dtau = torch.empty(H, C, device=device), torch.empty(H, device=device), torch.empty(1, device=device)
    wsb = lib.aimx_attn_pool_workspace_bytes(n, C, H, G)
    ws = torch.empty(wsb // 4 + 1, device=device)
    rp, col = P(plan.graph.rowptr), P(plan.graph.col)

    def fwd():
        assert lib.aimx_attn_pool_forward(P(x), C, n, C, P(W), P(b), P(tau), H, rp, col, G, P(pooled), P(attn),
                                          P(scores), _lib.stream_ptr(device)) == 0

    def bwd():
        assert lib.aimx_attn_pool_backward(P(x), C, n, C, P(W), P(tau), H, rp, col, G, P(attn), P(scores), P(dpool),
                                           None, P(dx), C, P(dW), P(db), P(dtau), P(ws), wsb,
                                           _lib.stream_ptr(device)) == 0
    fwd()
    tf, tb = graph_time_us(fwd), graph_time_us(bwd)
    bf = 4 * (n * C + 2 * H * n + G * C + H * C)
    bb = 4 * (2 * n * C + 2 * H * n + G * C + 2 * H * C)
    return {"atoms": n, "molecules": G, "C": C, "heads": H,
            "fwd": _bw("k_attn_fwd", bf, tf), "bwd": _bw("k_attn_bwd + partial reduce", bb, tb)}


MFMA_F32_PEAK_TFS = 157.3  # dense fp32 MFMA (v_mfma_f32_16x16x4_f32), MI355X_MICROARCH.md chip table


def step_flops(cfg, n_atoms, n_mols, emb=64, n_feat=4, mlp_blocks=2, ffn_blocks=3, heads=4):
    """fp32 GEMM flops of one train step (forward x 3 for forward + input and weight gradients).
    algorithmic: SURVEY §8d's count (the input projection over all h+1 chunks of F);
    executed: what the kernels multiply — the hop chunks >= 2 of F are exact zeros for reference
    inputs (targets never hop-offset, layers.py:154) and are skipped (DESIGN.md §3 'Empty hop
    chunks'), so the input projection contracts over 2·D."""
    H, h, D, T, L = cfg["hidden"], cfg["hops"], int(0.3 * cfg["hidden"]), cfg["tasks"], 3
    N, G = n_atoms, n_mols
    common = 2 * N * emb * n_feat * H + 2 * N * H * H + 2 * 2 * N * H * heads  # embed proj, concat, attn scores+sum
    head = 2 * G * (H * H + ffn_blocks * 2 * H * H + H * H + 2 * H * T)
    mlp = mlp_blocks * 2 * 2 * N * D * D
    alg = common + head + L * (2 * N * D * (h + 1) * 2 * D + mlp)
    exe = common + head + L * (2 * N * 2 * D * 2 * D + mlp)
    return 3 * alg, 3 * exe


def concat_gemm(n_atoms, hidden, device):
    """The largest single GEMM of the step, concat_self_other forward ([N, hidden] x [hidden, hidden]
    + bias, gnn.py:245-246), alone through the C ABI."""
    from aimx import ops
    x = torch.randn(n_atoms, hidden, device=device)
    W = torch.randn(hidden, hidden, device=device) * hidden ** -0.5
    b = torch.zeros(hidden, device=device)
    out = torch.empty(n_atoms, hidden, device=device)
    us = graph_time_us(lambda: ops.gemm_linear_fwd(x, hidden, W, b, out, hidden))
    fl = 2 * n_atoms * hidden * hidden
    tfs = fl / (us * 1e-6) / 1e12
    return {"kernel": "k_gemm (concat_self_other fwd)", "M": n_atoms, "N": hidden, "K": hidden, "flops": fl,
            "us_per_launch": round(us, 2), "achieved": round(tfs, 2), "unit": "TFLOP/s", "peak": MFMA_F32_PEAK_TFS,
            "frac": round(tfs / MFMA_F32_PEAK_TFS, 4)}


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return model, os.cpu_count(), affinity


def cpu_baseline(cfg, seconds=10.0, max_steps=40, one_thread_seconds=6.0):
    """Oracle CPU restatement of the reference train step (fwd+bwd+clip+Adam, dropout on): on the
    box's CPU share (min(16, cpu_count) threads: the box's cgroup quota is 16 CPUs' worth of time,
    `value`) and on 1 thread (BASELINE.md CPU-baseline plan item 3); the port/reference ratio comes
    from profiles/port_vs_reference.json (the reference itself only runs in the development
    container). (Round 4's extra figure on os.cpu_count() threads oversubscribed that quota 16x and
    measured the oversubscription, not the CPU; it is gone.)"""
    threads = min(16, os.cpu_count() or 1)
    res = _cpu_rate(cfg, threads, seconds, max_steps)
    res1 = _cpu_rate(cfg, 1, one_thread_seconds, 8)
    model, count, affinity = cpu_info()
    quota = None
    try:  # cgroup v2 CPU quota: "max period" or "<quota> <period>" (CPUs' worth of time)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    res["cgroup_cpu_quota"] = quota
    res.update({"value_1thread": res1["value"], "sample_1thread": res1["sample"], "cpu_model": model,
                "cpu_count": count, "cpu_affinity": affinity})
    pvr = os.path.join(ROOT, "profiles", "port_vs_reference.json")
    if os.path.exists(pvr):
        try:
            rec = json.load(open(pvr))
            res["port_vs_reference"] = {k: rec.get(k) for k in ("ratio_port_over_reference", "oracle_mol_per_s",
                                                                 "reference_mol_per_s", "threads", "cpu_model",
                                                                 "measured", "script")}
        except (OSError, ValueError):
            pass
    return res


def _cpu_rate(cfg, threads, seconds, max_steps):
    from oracle import model as om
    torch.set_num_threads(threads)
    mcfg = om.default_config(hidden_dim=cfg["hidden"], num_shells=cfg["hops"], output_dim=cfg["tasks"],
                             use_partial_charges=cfg["pc"])
    params = {k: v.requires_grad_() for k, v in om.seeded_params(mcfg, 0).items()}
    opt = torch.optim.Adam(params.values(), lr=2.5e-4)
    b = make_batches(cfg, 1, 4321, "cpu", pad=False)[0]
    af, edges, batch, tc, _, _, _ = b.model_args()

    def step():
        opt.zero_grad(set_to_none=True)
        out, _, _ = om.gnn_forward(params, mcfg, af, edges, batch, tc, training=True)
        loss = torch.nn.functional.l1_loss(out, b.targets)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params.values(), 1.0)
        opt.step()

    step()
    n, t0 = 0, time.perf_counter()
    while n < max_steps and (time.perf_counter() - t0) < seconds:
        step()
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(cfg["batch"] * n / dt, 1), "unit": "molecules/s", "cores": threads, "kind": "port",
            "sample": f"{n} train steps x {cfg['batch']} molecules ({cfg['source']}, hidden {cfg['hidden']}, "
                      f"{cfg['hops']} hops), oracle/model.py fp32 torch-CPU, {threads} threads"}


def eager_rate(cfg, device, batches_eager=4, steps=20, warmup=5, autograph=False, seed=777, ddp=False):
    """The drop-in (unchanged reference trainer) rate: a fresh model trained eagerly on unpadded
    resident batches — forward, L1 loss, backward, clip + Adam, one Python call per op as
    trainer.py:151-164 runs it (no graph). autograph: the same loop with aimx.autograph on (the
    model's forward and backward replayed per shape bucket, AIMX_AUTOGRAPH=1); the bucket's
    capture happens in the warm-up. ddp: the same loop on the model wrapped as the reference
    runner wraps it (DistributedDataParallel(find_unused_parameters=True), runner.py:703-707) over
    the initialised process group. A side measurement; never the metric `value`."""
    from aimx.optim import FusedAdam
    from models import L1Loss
    model = build_model(cfg, device)
    from aimx import autograph as ag
    if not autograph:
        ag.enable(model, False)  # autograph=True: the default drop-in behaviour (size-gated replay)
    opt = FusedAdam(model.parameters(), lr=2.5e-4, max_grad_norm=1.0)
    loss_fn = L1Loss()
    bs = make_batches(cfg, batches_eager, seed, device, pad=False)
    net = model
    if ddp:
        from torch.nn.parallel import DistributedDataParallel as DDP
        net = DDP(model, device_ids=[torch.device(device).index or 0], find_unused_parameters=True)

    def step(i):
        b = bs[i % len(bs)]
        opt.zero_grad(set_to_none=True)
        out, _, _ = net(*b.model_args())
        loss_fn(out, b.targets).backward()
        opt.step()
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    replayed = bool(autograph and ag.wanted(model.train(), bs[0].model_args()))
    del model, opt, bs, net
    torch.cuda.empty_cache()
    return {"value": round(cfg["batch"] * steps / dt, 1), "unit": "molecules/s", "ms_per_step": round(dt / steps * 1e3, 4),
            "steps": steps, "warmup": warmup,
            "mode": ("DistributedDataParallel(find_unused_parameters=True)-wrapped model over a world-size-"
                     f"{dist.get_world_size() if dist.is_initialized() else 1} process group, " if ddp else "")
            + ("eager loop as the unchanged trainer runs it, the default drop-in behaviour: the model's "
                     "forward/backward replayed per shape bucket by aimx.autograph when atoms x hidden <= "
                     f"{ag.MAX_WORK} (here: {'replayed' if replayed else 'eager launches'}), unpadded batches, "
                     "same step") if autograph else
            "eager, every operator launched from Python (AIMX_AUTOGRAPH=0), unpadded batches, same step"}


def rank_env(base, rank, world, port, addr="127.0.0.1"):
    """The environment of rank `rank` of a `world`-rank single-node job: what torchrun exports and
    the reference reads (main/utils.py:41-52: LOCAL_RANK and WORLD_SIZE select DDP and the device),
    plus RANK / LOCAL_WORLD_SIZE / MASTER_* for the process-group rendezvous (env://). One GPU per
    rank: rank r runs on cuda:r."""
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "ROLE_RANK": str(rank),
                "ROLE_WORLD_SIZE": str(world), "MASTER_ADDR": addr, "MASTER_PORT": str(port),
                "TORCHELASTIC_RUN_ID": "aimx-bench"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    return env


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _pdeathsig():
    """A preexec_fn for the rank processes: the kernel sends the rank SIGKILL when this launcher
    dies for any reason (prctl(PR_SET_PDEATHSIG)), so a launcher killed by the driver's timeout
    leaves no rank holding a GPU. libc's prctl is bound here, in the parent: the child (between fork
    and exec, before anything touches a GPU) only calls it."""
    import ctypes
    import signal
    prctl = ctypes.CDLL(None, use_errno=True).prctl
    parent = os.getpid()

    def setup():
        prctl(1, int(signal.SIGKILL))  # PR_SET_PDEATHSIG
        if os.getppid() != parent:  # the launcher died before the request took effect
            os._exit(1)
    return setup


DEFAULT_DEADLINE_S = 600.0


def resolve_deadline(gpus, given):
    """--deadline as given, else DEFAULT_DEADLINE_S for a multi-GPU run and none at one GPU."""
    if given is not None:
        return float(given)
    return DEFAULT_DEADLINE_S if gpus > 1 else 0.0


def exit_code(ddp_check, capture_error):
    """The command's status after the line is printed: 3 when data-parallel replicas diverged (the
    numbers are not those of a correct run); 0 otherwise — also when the RCCL all-reduce capture fell
    back to split graphs, which is a correct run of the split mode that the line labels as such."""
    if ddp_check is not None and not ddp_check["replicas_identical"]:
        print("bench: data-parallel replicas diverged (parameter checksums differ across ranks)", file=sys.stderr)
        return 3
    if capture_error is not None:
        print(f"bench: warning: the RCCL all-reduce capture fell back to split graphs ({capture_error}); "
              "the line reports the split-graph step", file=sys.stderr)
    return 0


def rank_watchdog(deadline_s):
    """Exit this rank with 124 once `deadline_s` seconds have passed (a daemon timer; a rank that
    finishes first never hears from it). A collective hung on a lost peer then ends the rank, and its
    launcher (torchrun, or launch_ranks) stops the others, instead of every rank waiting for the
    outer timeout. os._exit ends the process where it stands: nothing is exec'd."""
    import threading

    def expire():
        print(f"bench: rank {os.environ.get('RANK', '?')}: deadline of {deadline_s:g} s passed (hung collective?); "
              "exiting 124", file=sys.stderr, flush=True)
        os._exit(124)
    t = threading.Timer(deadline_s, expire)
    t.daemon = True
    t.start()
    return t


def launch_ranks(n, argv, poll_s=0.2, script=None, deadline_s=0.0, straggler_s=300.0):
    """`python bench.py --gpus N` without a launcher: start N rank processes of this same script
    (children, never an exec of this process) and wait for them. This process never touches the
    GPU. Rank 0's stdout is this command's stdout (the one JSON line); the others' stdout goes to
    stderr. The first rank to fail stops the rest, and its exit code is returned (a rank that dies
    would otherwise leave its peers waiting in a collective).

    No rank outlives the launcher or hangs it: SIGTERM / SIGINT / SIGHUP to the launcher are
    forwarded to every rank's process group (exit 128 + the signal), each rank gets a parent-death
    SIGKILL (_pdeathsig: a launcher killed outright takes its ranks with it), and the launcher stops
    every rank and exits 124 once `deadline_s` (> 0) has passed since the start, or `straggler_s`
    since the first rank finished cleanly while others still run (a peer hung in a collective)."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    got = []
    sigs = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)
    old = {sg: signal.signal(sg, lambda sig, frame: got.append(sig)) for sg in sigs}
    setup = _pdeathsig()
    t0 = time.time()
    first_ok = None
    rc = 0
    try:
        for r in range(n):
            procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv),
                                          env=rank_env(os.environ, r, n, port),
                                          stdout=None if r == 0 else sys.stderr.fileno(), start_new_session=True,
                                          preexec_fn=setup))
        while True:
            if got:
                rc = 128 + int(got[0])
                print(f"bench: launcher got signal {int(got[0])}; stopping every rank", file=sys.stderr)
                break
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                print(f"bench: a rank exited with {rc}; stopping the other ranks", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            now = time.time()
            if first_ok is None and any(c == 0 for c in codes):
                first_ok = now
            if deadline_s and now - t0 > deadline_s:
                rc = 124
                print(f"bench: deadline of {deadline_s:g} s passed; stopping every rank", file=sys.stderr)
                break
            if first_ok is not None and straggler_s and now - first_ok > straggler_s:
                rc = 124
                print(f"bench: ranks still running {straggler_s:g} s after a peer finished (hung in a "
                      "collective?); stopping them", file=sys.stderr)
                break
            time.sleep(poll_s)
    finally:
        if rc or len(procs) < n:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            grace = time.time() + 10
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, grace - time.time()))
                except subprocess.TimeoutExpired:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    p.wait()
        for sg, h in old.items():
            signal.signal(sg, h)
    return 128 - rc if rc < 0 else rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--pool", type=int, default=8, help="distinct resident batches cycled per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--roofline-only", action="store_true", help="only run the hop roofline launches (profiling)")
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="capture the whole train step in a HIP graph (static padded batches; default)")
    ap.add_argument("--no-graph", dest="graph", action="store_false", help="eager execution")
    ap.add_argument("--feed", default="resident", choices=["resident", "native", "stream"],
                    help="resident: a pool of batches already in HBM (the metric's `value`); native: every "
                         "step's batch is collated by the C++ batch builder from the molecule store and "
                         "copied host->device inside the timed region (PCIe-inclusive rate); stream: the same "
                         "from an HDF5 file in the reference's dataset format, read and decoded in C++ on a "
                         "prefetch thread (this rank's equal shard)")
    ap.add_argument("--stream-mols", type=int, default=200_000, help="molecules in the --feed stream file")
    ap.add_argument("--stream-path", default=None, help="--feed stream file (default: generated under $TMPDIR)")
    ap.add_argument("--feed-threads", type=int, default=8)
    ap.add_argument("--read-threads", type=int, default=None, help="HDF5 reader threads (default: --feed-threads)")
    ap.add_argument("--amp", action="store_true",
                    help="the reference's --mixed_precision path (trainer.py:134): the step runs under "
                         "torch.autocast('cuda', bfloat16) -> bf16 MFMA operands, fp32 accumulation in the GEMMs")
    ap.add_argument("--no-eager", action="store_true", help="skip the eager (no-graph) side measurement")
    ap.add_argument("--eager-steps", type=int, default=20)
    ap.add_argument("--ddp-world1", action="store_true",
                    help="A/B of the data-parallel step on one GPU: a world-size-1 RCCL group with the bucket "
                         "all-reduces kept (GradientSync always=True); --ddp-graph picks the mode")
    ap.add_argument("--ddp-graph", default="capture", choices=["capture", "split"],
                    help="data-parallel graph mode of GraphedTrainStep (capture: the RCCL all-reduces inside the "
                         "step graph; split: eager all-reduces between captured halves)")
    ap.add_argument("--quantum", type=int, default=None, help="atoms per static-layout bucket (A/B; default per config)")
    ap.add_argument("--deadline", type=float, default=None,
                    help="multi-GPU runs: every rank exits 124 this many seconds after it started (a hung "
                         "collective must not wait for an outer timeout), and a self-launched run (--gpus N without "
                         "torchrun) stops every rank then; 0: none. Default: %g s when --gpus > 1, none at one GPU"
                         % DEFAULT_DEADLINE_S)
    ap.add_argument("--straggler", type=float, default=300.0,
                    help="self-launched ranks: stop the others and exit 124 this many seconds after the first rank "
                         "finished cleanly (a peer hung in a collective)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse several ranks on one GPU")
    args = ap.parse_args()
    global QUANTUM_OVERRIDE
    QUANTUM_OVERRIDE = args.quantum

    if args.gpus < 1:
        print(f"bench: --gpus {args.gpus} must be >= 1", file=sys.stderr)
        sys.exit(2)
    args.deadline = resolve_deadline(args.gpus, args.deadline)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N`: start the N ranks here, before anything touches the GPU (the
        # launcher's own deadline a little after the ranks', so a rank's own exit is what it reports)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], deadline_s=args.deadline + 30 if args.deadline else 0.0,
                              straggler_s=args.straggler))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and args.deadline:
        rank_watchdog(args.deadline)
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to report a {world}-rank run as "
              f"{args.gpus} GPUs", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:  # rehearsal only (more ranks than GPUs): ranks share the box's GPUs
        if args.dist_backend == "nccl":
            print(f"bench: rank {rank} has LOCAL_RANK {local} but {ndev} visible GPU(s); RCCL needs one GPU "
                  "per rank (--dist-backend gloo rehearses several ranks on one GPU)", file=sys.stderr)
            sys.exit(2)
        local = local % ndev
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    cfg = CONFIGS[args.config]
    torch.manual_seed(1234 + rank)

    feeder = None
    if args.feed == "native":
        feeder = native_feeder(cfg, 1234 + rank, device, args.feed_threads, args.graph)
        batches = [next(feeder)]
    elif args.feed == "stream":
        feeder = stream_feeder(cfg, rank, world, device, args.feed_threads, args.graph, args.stream_mols,
                               args.stream_path, read_threads=args.read_threads)
        batches = [next(feeder)]
    else:
        # one GPU: one captured graph per 256-atom bucket of the pool; data parallel: one shape for all
        # (every rank must capture and replay the same graphs' collectives in step)
        batches = make_batches(cfg, args.pool, 1234 + rank, device, pad=args.graph,
                               buckets=world == 1 and not args.ddp_world1)
    if args.roofline_only:
        print(json.dumps(hop_roofline(make_batches(cfg, 1, 99, device)[0], cfg["hops"], device, cfg["hidden"])))
        return

    from aimx.optim import FusedAdam
    from utils.distributed import GradientSync
    model = build_model(cfg, device)
    B = cfg["batch"]
    from models import L1Loss
    loss_fn = L1Loss()  # the reference criterion (nn.L1Loss, trainer.py:34) as one fused launch each way

    sync = None
    if world > 1:
        # DDP-equivalent bucketed all-reduce (reference runner.py:703-707); the unused
        # long_range_projection (gnn.py:146) takes no part, as under find_unused_parameters
        sync = GradientSync(model.parameters(), unused=model.unused_parameters())
    elif args.ddp_world1:
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=device)
        sync = GradientSync(model.parameters(), unused=model.unused_parameters(), always=True)
    opt = FusedAdam(model.parameters(), lr=2.5e-4, max_grad_norm=1.0)  # clip(1.0) + Adam, trainer.py:163-164
    graphed = None
    pad_mols_used = "/".join(str(v) for v in sorted({b.num_graphs - B for b in batches})) if args.graph else "0"
    if args.graph:
        # Whole-step HIP-graph capture on static padded inputs (aimx.train.GraphedTrainStep): forward,
        # backward, the bucketed RCCL all-reduces overlapped with the backward (world > 1), clip and
        # Adam; each timed step copies a fresh resident batch into the static inputs and replays.
        from aimx.train import GraphedTrainStep
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.amp):  # captured in the context
            graphed = GraphedTrainStep(model, loss_fn, opt, batches[0], n_real=B, sync=sync, ddp_graph=args.ddp_graph,
                                       max_layouts=8 if sync is None else 1)
            graphed.prepare(batches)

        def step(i):
            graphed(next(feeder) if feeder is not None else batches[i % len(batches)])
    else:
        def step(i):
            b = next(feeder) if feeder is not None else batches[i % len(batches)]
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.amp):
                out, _, _ = model(*b.model_args())
                loss = loss_fn(out[:B], b.targets[:B])
            loss.backward()
            if sync is not None:
                sync.finish()
            opt.step()

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if feeder is not None:
        feeder.reset_stats()  # the feed's per-stage times over the timed steps only
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    feed_stats = None
    if feeder is not None:
        feed_stats = feeder.stats()
        feeder.close()
    ddp_check = None
    if sync is not None:
        # self-verification of the data-parallel run (every rank takes part): replicas bit-identical
        # after the timed steps, and the collectives' own cost per step
        from utils.distributed import replica_checksums
        identical, local, mx, mn = replica_checksums(list(model.parameters()), device)
        ar_us = sync.time_allreduce(iters=20)
        t = torch.tensor([ar_us], device=device, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ddp_check = {"replicas_identical": identical, "param_checksum_max": mx, "param_checksum_min": mn,
                     "allreduce_us_per_step": round(float(t.item()), 2),
                     "allreduce_note": "every bucket's all-reduce alone, back to back (HIP events on the "
                                       "collectives' stream), max over ranks; inside the timed steps they "
                                       "overlap the backward"}
    from aimx import _lib as alib
    # a clustered head wait gave up on ANY rank: the run is invalid (max over ranks)
    tmo = alib.head_sync_flag(device).reshape(1)
    if world > 1:
        dist.all_reduce(tmo, op=dist.ReduceOp.MAX)
    head_timeout = bool(tmo.item() != 0)
    if head_timeout:
        print("bench: a clustered head launch timed out; results invalid", file=sys.stderr)
    atoms = sum(getattr(b, "real_atoms", b.num_atoms) for b in batches) / len(batches)
    edges = sum(getattr(b, "real_edges", b.edges.shape[0]) for b in batches) / len(batches)
    mol = cfg["batch"] * world * args.steps
    value = mol / dt

    eager = None
    if rank == 0 and world == 1 and args.graph and feeder is None and not args.no_eager and not args.amp:
        # the same resident batches as the graphed loop, unpadded
        eager = eager_rate(cfg, device, batches_eager=args.pool, steps=args.eager_steps, seed=1234)
        eager["autograph"] = eager_rate(cfg, device, batches_eager=args.pool, steps=args.eager_steps, seed=1234,
                                        autograph=True)
        if dist.is_initialized():  # --ddp-world1: the reference's DDP wrapping over the autograph
            eager["ddp_wrapped"] = eager_rate(cfg, device, batches_eager=args.pool, steps=args.eager_steps,
                                              seed=1234, autograph=True, ddp=True)
    roof = extra = None
    if rank == 0 and not args.no_roofline:
        del batches
        torch.cuda.empty_cache()
        probe = make_batches(cfg, 1, 99, device)[0]
        roof = hop_roofline(probe, cfg["hops"], device, cfg["hidden"])
        fl_alg, fl_exe = step_flops(cfg, atoms, cfg["batch"])
        step_s = dt / args.steps
        extra = {
            "hop_in_step": hop_in_step(probe, cfg["hops"], cfg["hidden"], device),
            "attn_in_step": attn_in_step(probe, cfg["hidden"], device),
            "mfma": {"bound": "mfma", "unit": "TFLOP/s", "peak": MFMA_F32_PEAK_TFS,
                     "step_flops_algorithmic": fl_alg, "step_flops_executed": fl_exe,
                     "achieved_step_executed": round(fl_exe / step_s / 1e12, 2),
                     "frac_step_executed": round(fl_exe / step_s / 1e12 / MFMA_F32_PEAK_TFS, 4),
                     "achieved_step_algorithmic": round(fl_alg / step_s / 1e12, 2),
                     "note": "whole-step rate over the whole step time (GEMMs + every HBM-bound kernel); "
                             "executed skips the exact-zero hop chunks (step_flops)",
                     "largest_gemm": concat_gemm(int(atoms), cfg["hidden"], device)},
        }
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg)
    if rank == 0:
        line = {
            "metric": "molecules/sec fwd+bwd on QM9-shaped batches; achieved HBM GB/s on scatter-add hop",
            "value": round(value, 1), "unit": "molecules/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16 GEMM operands, fp32 accumulation and tensors (AMP)" if args.amp else "fp32",
            "data": "synthetic",
            "config": {"workload": f"{args.config}: " + ("QM9-shaped" if cfg["source"] == "qm9" else "40-atom synthetic")
                       + f", hidden {cfg['hidden']}, {cfg['hops']} hops, {cfg['tasks']} task(s), attention pool, "
                       "train step fwd+bwd+clip+Adam, dropout 0.05"
                       + (f", HIP-graph replay of padded static batches (+{pad_mols_used} padding molecules of"
                          " <= 64 atoms, excluded from the loss; "
                          + (f"{graphed.layouts} captured layouts: {layout_quantum(cfg)}-atom buckets)" if sync is None
                             else "one layout)") if args.graph else ", eager"),
                       "feed": ("resident pool of %d batches in HBM" % args.pool if feeder is None else
                                "native C++ collate + pinned H2D per step (PCIe-inclusive; not the metric value)"
                                if args.feed == "native" else
                                f"HDF5 stream of {args.stream_mols} molecules (reference format), C++ read + "
                                "decode + collate + pinned H2D per step (PCIe-inclusive; not the metric value)"),
                       "global_batch": cfg["batch"] * world, "per_gpu_batch": cfg["batch"],
                       "mean_atoms_per_batch": round(atoms, 1), "mean_edges_per_batch": round(edges, 1),
                       "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if extra is not None:
            line.update(extra)
        if eager is not None:
            line["eager"] = eager
        if feed_stats is not None:
            line["feed_ms_per_batch"] = feed_stats
            if graphed is not None:  # steps (warmup included) whose batch was over the static capacity
                line["graph_eager_steps"] = graphed.eager_steps
        if STREAM_INFO:
            line["stream_file"] = dict(STREAM_INFO)
        if sync is not None:
            line["ddp"] = {"world_size_reported": dist.get_world_size(), "backend": dist.get_backend(),
                           "graph_mode": graphed.mode if graphed is not None else "eager",
                           "capture_fallback": graphed is not None and graphed.capture_error is not None,
                           "capture_error": (str(graphed.capture_error)[:300] if graphed is not None and
                                             graphed.capture_error is not None else None),
                           "rccl": getattr(sync.comm, "info", None),
                           "buckets": len(sync.buckets),
                           "bucket_mb": [round(sum(p.numel() for p in bk) * 4 / 2 ** 20, 3) for bk in sync.buckets],
                           **ddp_check}
        if cpu is not None:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        if head_timeout:
            line["invalid"] = "clustered head wait timed out"
        if ddp_check is not None and not ddp_check["replicas_identical"]:
            line["invalid"] = "data-parallel replicas diverged"
        print(json.dumps(line), flush=True)
    # a data-parallel run that diverged is reported above and then fails the command (every rank knows
    # it). An RCCL capture that fell back to split graphs is a valid measurement of the split mode: the
    # line says so (ddp.graph_mode "split", ddp.capture_error) and the command succeeds
    rc = exit_code(ddp_check, graphed.capture_error if graphed is not None else None)
    if dist.is_initialized():
        dist.destroy_process_group()
    if rc:
        sys.exit(rc)


if __name__ == "__main__":
    main()
