"""Native batch feed: the C++ batch builder (libaimx_host.so, include/aimx_host.h) behind Python.

Replaces the reference's host input path for the hot path:
  * src/datasets/features.py:82-150  multi-hop BFS pair lists (per molecule)
  * src/datasets/molecular.py:339-458 MyBatch.from_data_list (collate)
  * trainer.py:123-131 per-tensor `.to(device)` copies
with one native plan+write per batch straight into a pinned host blob in DeviceBatch layout and ONE
async host->device copy of that blob on a copy stream. `BatchFeeder` keeps `depth` batches in
flight from a background thread (ctypes releases the GIL inside the native calls), so collation
and the PCIe copy overlap the GPU step.

Everything here is bit-identical to aimx.data (the Python restatement) and to the reference's own
BFS + collate fixtures (tests/test_host_collate.py).
"""
from __future__ import annotations

import atexit
import ctypes
import os
import queue
import threading
import weakref

import numpy as np
import torch

from . import data as adata

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libaimx_host.so")

c_i64, c_i32, c_ptr = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
_ERR = {-1: "invalid argument", -2: "capacity too small", -3: "out of host memory", -4: "write without a plan"}


class HostError(RuntimeError):
    code = 0  # the aimx_host status (-2: a batch larger than the caller's capacity)


class CollateOut(ctypes.Structure):
    _fields_ = [("feat", c_ptr * 8), ("edges", c_ptr), ("batch", c_ptr), ("total_charges", c_ptr),
                ("targets", c_ptr), ("n_atoms", c_ptr), ("n_max", c_i64), ("e_max", c_i64), ("pad_mols", c_i32)]


_lib = None


def load_host():
    """Load libaimx_host.so (built by `make -C aimnet-x2d_amd/csrc`); raises HostError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(HOST_LIB_PATH):
        raise HostError(f"{HOST_LIB_PATH} not built (run make -C aimnet-x2d_amd/csrc)")
    lib = ctypes.CDLL(HOST_LIB_PATH)
    lib.aimx_host_version.restype = ctypes.c_char_p
    lib.aimx_bfs_multi_hop.restype = c_i64
    lib.aimx_bfs_multi_hop.argtypes = [c_i32, c_ptr, c_i64, c_i32, c_ptr, c_i64, c_ptr]
    lib.aimx_store_create.restype = c_i32
    lib.aimx_store_create.argtypes = [c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_i32, c_ptr, c_i32, c_ptr, c_i32, c_i32,
                                      ctypes.POINTER(c_ptr)]
    lib.aimx_store_create_hops.restype = c_i32
    lib.aimx_store_create_hops.argtypes = [c_i64, c_ptr, c_ptr, c_i32, c_i32, c_ptr, c_ptr, c_ptr, c_i32, c_ptr,
                                           ctypes.POINTER(c_ptr)]
    lib.aimx_store_destroy.argtypes = [c_ptr]
    lib.aimx_store_num_molecules.restype = c_i64
    lib.aimx_store_num_molecules.argtypes = [c_ptr]
    lib.aimx_store_num_atoms.restype = c_i64
    lib.aimx_store_num_atoms.argtypes = [c_ptr, c_i64]
    lib.aimx_store_atom_counts.restype = c_i32
    lib.aimx_store_atom_counts.argtypes = [c_ptr, c_ptr]
    lib.aimx_collator_create.restype = c_i32
    lib.aimx_collator_create.argtypes = [c_i32, c_i32, ctypes.POINTER(c_ptr)]
    lib.aimx_collator_destroy.argtypes = [c_ptr]
    lib.aimx_collate_plan.restype = c_i32
    lib.aimx_collate_plan.argtypes = [c_ptr, c_ptr, c_ptr, c_i64, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]
    lib.aimx_collate_write.restype = c_i32
    lib.aimx_collate_write.argtypes = [c_ptr, ctypes.POINTER(CollateOut)]
    lib.aimx_csr_host_build.restype = c_i32
    lib.aimx_csr_host_build.argtypes = [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i32] + [c_ptr] * 6
    lib.aimx_collate_csr.restype = c_i32
    lib.aimx_collate_csr.argtypes = [c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i32] + [c_ptr] * 6
    _lib = lib
    return lib


def _check(rc, what):
    if rc < 0:
        e = HostError(f"aimx_host {what}: {_ERR.get(int(rc), rc)}")
        e.code = int(rc)
        raise e
    return rc


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def bfs_multi_hop(n_atoms, bonds, max_hops):
    """Native restatement of features.py:97-150; same return shape as aimx.data.bfs_multi_hop."""
    lib = load_host()
    b = np.ascontiguousarray(np.asarray(bonds).reshape(-1, 2), np.int32)
    counts = np.zeros(max(max_hops, 1), np.int64)
    cap = max(64, 4 * n_atoms * max(max_hops, 1))
    while True:
        pairs = np.empty((cap, 2), np.int32)
        tot = _check(lib.aimx_bfs_multi_hop(n_atoms, _p(b), b.shape[0], max_hops, pairs.ctypes.data, cap,
                                            counts.ctypes.data), "bfs")
        if tot <= cap:
            break
        cap = tot
    out, o = [], 0
    for h in range(max_hops):
        c = int(counts[h])
        out.append(pairs[o:o + c].T.copy())
        o += c
    return out


class HostStore:
    """Molecule records in native memory (the fields collate reads from each reference Data object).

    precompute_hops > 0 caches every molecule's hop pairs at creation (the reference stores
    multi_hop_edges in its datasets, features.py:416-431); 0 runs the BFS inside each collate."""

    def __init__(self, n_atoms, bonds_per_mol, feats, targets=None, total_charge=None, precompute_hops=0,
                 threads=4):
        lib = load_host()
        n_atoms = np.asarray(n_atoms, np.int64)
        nb = np.array([len(b) for b in bonds_per_mol], np.int64)
        self._atom_ptr = np.concatenate([[0], np.cumsum(n_atoms)]).astype(np.int64)
        self._bond_ptr = np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)
        bonds = (np.concatenate([np.asarray(b, np.int32).reshape(-1, 2) for b in bonds_per_mol])
                 if len(bonds_per_mol) else np.zeros((0, 2), np.int32))
        self._init(lib, n_atoms.shape[0], bonds, feats, targets, total_charge, precompute_hops, threads)

    @classmethod
    def from_arrays(cls, atom_ptr, bond_ptr, bonds, feats, targets=None, total_charge=None, precompute_hops=0,
                    threads=4):
        s = cls.__new__(cls)
        s._atom_ptr = np.ascontiguousarray(atom_ptr, np.int64)
        s._bond_ptr = np.ascontiguousarray(bond_ptr, np.int64)
        s._init(load_host(), s._atom_ptr.shape[0] - 1, bonds, feats, targets, total_charge, precompute_hops, threads)
        return s

    @classmethod
    def from_qm9_asset(cls, asset, precompute_hops=0, threads=4):
        bonds = np.stack([asset.bi, asset.bj], 1)
        return cls.from_arrays(asset.atom_off, asset.bond_off, bonds, asset.feats, asset.targets,
                               asset.total_charge, precompute_hops, threads)

    @classmethod
    def from_molecules(cls, mols, targets=None, total_charge=None, precompute_hops=0, threads=4):
        """mols: list of (n_atoms, bonds [B,2], feats [n,F]) as produced by aimx.synth."""
        feats = (np.concatenate([np.asarray(m[2]).reshape(m[0], -1) for m in mols])
                 if mols else np.zeros((0, len(adata.FEATURE_KEYS)), np.int32))
        return cls([m[0] for m in mols], [m[1] for m in mols], feats, targets, total_charge, precompute_hops, threads)

    @classmethod
    def from_handle(cls, handle, n_feat, n_tasks):
        """Adopt a native store created elsewhere (e.g. aimx_h5_read_store); destroyed with this object."""
        lib = load_host()
        s = cls.__new__(cls)
        s._lib, s._h = lib, handle
        s.n_feat, s.n_tasks = int(n_feat), int(n_tasks)
        s.n_mols = int(lib.aimx_store_num_molecules(handle))
        s.n_atoms = np.empty(s.n_mols, np.int64)
        _check(lib.aimx_store_atom_counts(handle, s.n_atoms.ctypes.data), "store_atom_counts")
        return s

    @classmethod
    def from_hop_lists(cls, n_atoms, hops_per_mol, feats, targets=None, total_charge=None):
        """A store from precomputed hop arrays (the reference's multi_hop_edges: per molecule a list
        of int [2, E_h] arrays, one per hop) instead of bonds."""
        lib = load_host()
        n_atoms = np.asarray(n_atoms, np.int64)
        n_mols = n_atoms.shape[0]
        H = len(hops_per_mol[0]) if n_mols else 1
        lens = np.array([[np.asarray(e).reshape(2, -1).shape[1] for e in hops] for hops in hops_per_mol],
                        np.int64).reshape(n_mols, H)
        hop_ptr = np.concatenate([[0], np.cumsum(lens.reshape(-1))]).astype(np.int64)
        pairs = (np.concatenate([np.asarray(e).reshape(2, -1).T for hops in hops_per_mol for e in hops])
                 if n_mols else np.zeros((0, 2)))
        pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        atom_ptr = np.concatenate([[0], np.cumsum(n_atoms)]).astype(np.int64)
        feats = np.ascontiguousarray(feats, np.int32)
        n_feat = feats.shape[1] if feats.ndim == 2 else len(adata.FEATURE_KEYS)
        tg = None if targets is None else np.ascontiguousarray(np.asarray(targets, np.float32).reshape(n_mols, -1))
        tc = None if total_charge is None else np.ascontiguousarray(total_charge, np.float32)
        h = c_ptr()
        _check(lib.aimx_store_create_hops(n_mols, atom_ptr.ctypes.data, _p(feats), n_feat, H, hop_ptr.ctypes.data,
                                          _p(pairs), _p(tg), 0 if tg is None else tg.shape[1], _p(tc),
                                          ctypes.byref(h)), "store_create_hops")
        return cls.from_handle(h, n_feat, 0 if tg is None else tg.shape[1])

    def _init(self, lib, n_mols, bonds, feats, targets, total_charge, precompute_hops, threads):
        self._lib = lib
        bonds = np.ascontiguousarray(np.asarray(bonds).reshape(-1, 2), np.int32)
        feats = np.ascontiguousarray(feats, np.int32)
        self.n_feat = feats.shape[1] if feats.ndim == 2 else len(adata.FEATURE_KEYS)
        tg = None if targets is None else np.ascontiguousarray(np.asarray(targets, np.float32).reshape(n_mols, -1))
        self.n_tasks = 0 if tg is None else tg.shape[1]
        tc = None if total_charge is None else np.ascontiguousarray(total_charge, np.float32)
        h = c_ptr()
        _check(lib.aimx_store_create(n_mols, self._atom_ptr.ctypes.data, self._bond_ptr.ctypes.data, _p(bonds),
                                     _p(feats), self.n_feat, _p(tg), self.n_tasks, _p(tc), int(precompute_hops),
                                     int(threads), ctypes.byref(h)), "store_create")
        self._h = h
        self.n_mols = int(n_mols)
        self.n_atoms = np.diff(self._atom_ptr)

    def __len__(self):
        return self.n_mols

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.aimx_store_destroy(h)
            self._h = None


class HostCollator:
    """One native collator (persistent worker pool). Not thread-safe: one batch at a time."""

    def __init__(self, max_hops, threads=4, csr=True):
        self._lib = load_host()
        h = c_ptr()
        _check(self._lib.aimx_collator_create(int(max_hops), int(threads), ctypes.byref(h)), "collator_create")
        self._h = h
        self.max_hops = int(max_hops)
        # collate_blob also builds the batch's CSR views for a model of max_hops hops (csr=False: not)
        self.csr_hops = self.max_hops if csr else 0
        self._layouts = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.aimx_collator_destroy(h)
            self._h = None

    def plan(self, store, idx):
        self._idx = np.ascontiguousarray(idx, np.int64)
        n, e = c_i64(), c_i64()
        _check(self._lib.aimx_collate_plan(self._h, store._h, _p(self._idx), self._idx.shape[0], ctypes.byref(n),
                                           ctypes.byref(e)), "collate_plan")
        self._store = store
        return int(n.value), int(e.value)

    def write(self, feat_ptrs, edges, batch, total_charges=None, targets=None, n_atoms=None, n_max=0, e_max=0,
              pad_mols=0):
        o = CollateOut()
        for k, p in enumerate(feat_ptrs):
            o.feat[k] = p
        o.edges, o.batch, o.total_charges, o.targets, o.n_atoms = edges, batch, total_charges, targets, n_atoms
        o.n_max, o.e_max, o.pad_mols = int(n_max), int(e_max), int(pad_mols)
        _check(self._lib.aimx_collate_write(self._h, ctypes.byref(o)), "collate_write")

    def collate(self, store, idx):
        """Numpy arrays in aimx.data.collate's format (plus targets / total charges)."""
        n, e = self.plan(store, idx)
        g = self._idx.shape[0]
        feats = np.empty((store.n_feat, n), np.int64)
        edges = np.empty((e, 2), np.int64)
        batch = np.empty(n, np.int64)
        tc = np.empty(g, np.float32)
        tg = np.empty((g, max(store.n_tasks, 1)), np.float32)
        na = np.empty(g, np.int64)
        self.write([feats[k].ctypes.data for k in range(store.n_feat)], edges.ctypes.data, batch.ctypes.data,
                   tc.ctypes.data, tg.ctypes.data if store.n_tasks else None, na.ctypes.data)
        return {"edges": edges, "feats": feats.T.copy(), "batch": batch, "n_atoms": na, "total_charges": tc,
                "targets": tg[:, :store.n_tasks]}

    def blob_layout(self, nr, er, gr, t):
        """(layout, nbytes) of a blob of these row counts (cached: the same every padded batch)."""
        key = (nr, er, gr, t)
        hit = self._layouts.get(key)
        if hit is None:
            hit = self._layouts[key] = adata.blob_layout(adata.batch_fields(nr, er, gr, max(t, 1), self.csr_hops))
        return hit

    def collate_blob(self, store, idx, pinned=True, n_max=0, e_max=0, pad_mols=0, n_tasks=None, out=None):
        """Plan + write one batch into a (pinned) host byte tensor in DeviceBatch layout (`out`: an
        existing one of the right size, e.g. a feeder ring slot). Returns (blob uint8 tensor,
        layout, G_rows, N_rows, real (G, N, E))."""
        n, e = self.plan(store, idx)
        g = self._idx.shape[0]
        pad = n_max > 0
        nr, er, gr = (n_max, e_max, g + pad_mols) if pad else (n, e, g)
        t = store.n_tasks if n_tasks is None else n_tasks
        layout, nbytes = self.blob_layout(nr, er, gr, t)
        if out is not None:
            if out.numel() != nbytes:
                raise HostError(f"collate_blob: out has {out.numel()} bytes, the batch needs {nbytes}")
            blob = out
        else:
            blob = torch.empty(nbytes, dtype=torch.uint8, pin_memory=pinned)
        base = blob.data_ptr()
        ptr = [base + o for o, _, _ in layout]
        if t == 0:  # no targets in the store: zero the target field
            o, dt, shape = layout[-1]
            blob[o:o + int(np.prod(shape)) * 4].zero_()
        self.write(ptr[:4], ptr[4], ptr[5], ptr[6], ptr[7] if t else None, None, n_max if pad else 0,
                   e_max if pad else 0, pad_mols if pad else 0)
        if self.csr_hops > 0:  # the step's CSR views ride in the same blob (one H2D copy)
            _check(self._lib.aimx_collate_csr(self._h, ptr[4], er, ptr[5], nr, gr, self.csr_hops, *ptr[8:14]),
                   "collate_csr")
        return blob, layout, gr, nr, (g, n, e)


def static_capacity(collator, store, index_batches, atoms_slack=64, edges_slack=256, least_pad_mols=8):
    """Static shapes (n_max, e_max, pad_mols) for a padded BatchFeeder from sample index batches:
    the largest sampled atom / edge counts plus one standard deviation of them plus a fixed slack,
    and padding molecules of at most 64 atoms for batches down to 3 deviations under the smallest
    sample. A later batch that does not fit is handed out unpadded (BatchFeeder, stats()
    'overflow') and stepped eagerly (GraphedTrainStep): for counts near normal that is about one
    batch in 10^4 with 256 samples, so the margin stays a few tenths of a percent of compute
    instead of the 5-8 % a proportional margin costs."""
    sz = np.array([collator.plan(store, idx) for idx in index_batches], np.float64)
    if sz.size == 0:
        raise ValueError("static_capacity: no sample batches")
    n_sd, e_sd = sz.std(0)
    n_max = int(sz[:, 0].max() + n_sd) + atoms_slack
    e_max = int(sz[:, 1].max() + e_sd) + edges_slack
    pm = adata.pad_mols_for(n_max, max(int(sz[:, 0].min() - 3 * n_sd), 0), 64, least_pad_mols)
    return n_max, e_max, pm


class _Slot:
    """One ring entry of a static-shape BatchFeeder: pinned host blob, device blob, the DeviceBatch
    views over the device blob (built once), and the events that guard their reuse."""
    __slots__ = ("host", "dev", "batch", "h2d", "released", "index", "refs", "out")

    def __init__(self, nbytes, layout, gr, nr, hops, device):
        self.host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.batch = adata.DeviceBatch.from_blob(self.dev, layout, gr, nr, hops)
        self.h2d = torch.cuda.Event()       # the copy out of `host` is done (host reuse)
        self.released = torch.cuda.Event()  # the consumer's work on the batch is enqueued before it
        self.index = -1                     # item last held
        self.refs = None                    # reference count of `batch` while only the ring holds it
        self.out = False                    # handed to the consumer, `released` not yet recorded


_LIVE_FEEDERS = weakref.WeakSet()


@atexit.register
def _close_feeders():
    """Stop every feeder thread before interpreter teardown: a daemon thread still inside the
    native collate or an H2D enqueue while the process exits races the runtime's own teardown."""
    for f in list(_LIVE_FEEDERS):
        f.close()


class BatchFeeder:
    """Background native collation + async H2D copies, `depth` batches ahead of the consumer.

    batches: iterable of molecule-index arrays into `store`, or of (store, index array) pairs (a
    stream whose chunks are separate stores, aimx.h5.HDF5MolecularStream.batches; `store` may then
    be None). Yields DeviceBatch objects whose copy has been enqueued on the feeder's copy stream;
    the consumer's current stream waits on it (event), so the step never reads a half-copied batch
    and never blocks the host on the copy. Padding to static shapes (n_max/e_max/pad_mols) makes the
    batches replayable by one captured HIP graph.

    ring=True (static shapes only) keeps a ring of pinned host / device blobs with their batch views
    built once, so a batch costs one native collate (the pool's threads, GIL released), one async
    copy and two events, and no allocation. It is for consumers that COPY each batch before asking
    for the next one (GraphedTrainStep copies it into its static inputs): a slot is written again
    once its DeviceBatch object is referenced by nothing outside the ring (a consumer that keeps
    batch objects, e.g. list(feeder), makes the ring grow instead) and, on the device, after the
    consumer's work on it (its stream records `released` when it asks for the next batch) — but a
    kept tensor VIEW of a batch (batch.targets appended for an epoch metric) is not seen, and its
    contents change when the slot is refilled. By default (ring=False) every batch has a blob of
    its own, so anything kept stays valid.
    """

    def __init__(self, store, index_batches, max_hops, device, depth=3, threads=4, n_max=0, e_max=0, pad_mols=0,
                 ring=False):
        self.ring = bool(ring)
        self.store, self.device = store, torch.device(device)
        self.collator = HostCollator(max_hops, threads)
        self.pad = (n_max, e_max, pad_mols)
        self.stream = torch.cuda.Stream(self.device)
        self._q = queue.Queue(maxsize=depth)
        self._it = iter(index_batches)
        self._stop = False
        self._err = None
        self._ring = []           # static shapes: _Slot list (grows while the consumer keeps batches)
        self._next_slot = 0
        self._last = None         # the slot handed out last (released at the next request)
        # seconds spent per stage (feeder thread: next index batch / waiting for a ring slot's last
        # copy / native collate / H2D enqueue / batch views / waiting for queue room; consumer:
        # waiting for a batch), and counts
        self.reset_stats()
        self._th = threading.Thread(target=self._run, daemon=True)
        self._th.start()
        _LIVE_FEEDERS.add(self)

    def reset_stats(self):
        """Zero the stage times in place (the feeder thread keeps updating the same dict)."""
        if not hasattr(self, "times"):
            self.times = {}
        for k in ("source", "slot_wait", "collate", "h2d", "views", "put_wait", "get_wait"):
            self.times[k] = 0.0
        self.times["batches"] = 0
        self.times["overflow"] = 0  # static shapes: batches over capacity, handed out unpadded

    def _slot(self, nbytes, layout, gr, nr):
        """A ring slot free for the next batch: the oldest one nothing else references, else a new one."""
        import sys
        n = len(self._ring)
        for k in range(n):
            sl = self._ring[(self._next_slot + k) % n]
            if not sl.out and sys.getrefcount(sl.batch) <= sl.refs and sl.dev.numel() == nbytes:
                self._next_slot = (self._next_slot + k + 1) % n
                return sl
        sl = _Slot(nbytes, layout, gr, nr, self.collator.csr_hops, self.device)
        self._ring.insert(self._next_slot, sl)
        self._next_slot = (self._next_slot + 1) % len(self._ring)
        sl.refs = sys.getrefcount(sl.batch)
        return sl

    def _run(self):
        import time
        T = self.times
        static = self.pad[0] > 0
        use_ring = static and self.ring
        try:
            it = iter(self._it)
            while True:
                t0 = time.perf_counter()
                try:
                    item = next(it)
                except StopIteration:
                    break
                if self._stop:
                    break
                t1 = time.perf_counter()
                store, idx = item if isinstance(item, tuple) else (self.store, item)
                tc = t1
                sl = None
                if use_ring:
                    nr, er, gr = self.pad[0], self.pad[1], len(idx) + self.pad[2]
                    t = store.n_tasks
                    layout, nbytes = self.collator.blob_layout(nr, er, gr, t)
                    sl = self._slot(nbytes, layout, gr, nr)
                    if sl.index >= 0:
                        sl.h2d.synchronize()  # the pinned blob's previous copy has left it
                    tc = time.perf_counter()
                    T["slot_wait"] += tc - t1
                    try:
                        blob, layout, gr, nr, real = self.collator.collate_blob(store, idx, True, *self.pad,
                                                                                out=sl.host)
                    except HostError as e:
                        if e.code != -2:
                            raise
                        sl = None  # larger than the static capacity: this batch goes out unpadded
                    t2 = time.perf_counter()
                if sl is not None:
                    with torch.cuda.stream(self.stream):
                        if sl.index >= 0:
                            self.stream.wait_event(sl.released)
                        sl.dev.copy_(sl.host, non_blocking=True)
                        sl.h2d.record(self.stream)
                    sl.index += 1
                    t3 = time.perf_counter()
                    b = sl.batch
                    ev, keep = sl.h2d, sl
                else:
                    blob = None
                    if static and not use_ring:  # padded into a blob of its own
                        try:
                            blob, layout, gr, nr, real = self.collator.collate_blob(store, idx, True, *self.pad)
                        except HostError as e:
                            if e.code != -2:
                                raise
                    if blob is None:  # unpadded, or over the static capacity
                        if static:
                            T["overflow"] += 1
                        blob, layout, gr, nr, real = self.collator.collate_blob(store, idx, True)
                    t2 = time.perf_counter()
                    with torch.cuda.stream(self.stream):
                        dev = blob.to(self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    t3 = time.perf_counter()
                    b = adata.DeviceBatch.from_blob(dev, layout, gr, nr, self.collator.csr_hops)
                    keep = blob
                b.real_graphs, b.real_atoms, b.real_edges = real
                t4 = time.perf_counter()
                self._q.put((b, ev, keep))
                t5 = time.perf_counter()
                T["source"] += t1 - t0
                T["collate"] += t2 - tc
                T["h2d"] += t3 - t2
                T["views"] += t4 - t3
                T["put_wait"] += t5 - t4
                T["batches"] += 1
        except Exception as exc:  # surfaced to the consumer
            self._err = exc
        self._q.put(None)

    def stats(self):
        """Milliseconds per batch of each stage (see reset_stats), and the ring size."""
        n = max(self.times["batches"], 1)
        return {k: round(v * 1e3 / n, 4) for k, v in self.times.items() if k not in ("batches", "overflow")} | \
            {"batches": self.times["batches"], "overflow": self.times["overflow"], "ring": len(self._ring)}

    def __iter__(self):
        return self

    def __next__(self):
        import time
        cur = torch.cuda.current_stream(self.device)
        if self._last is not None:  # the consumer's work on the previous batch is enqueued
            self._last.released.record(cur)
            self._last.out = False
            self._last = None
        t0 = time.perf_counter()
        item = self._q.get()
        self.times["get_wait"] += time.perf_counter() - t0
        if item is None:
            if self._err is not None:
                raise self._err
            raise StopIteration
        b, ev, keep = item
        cur.wait_event(ev)
        if isinstance(keep, _Slot):
            keep.out = True
            self._last = keep
        else:
            b._host_blob = keep  # keep the pinned source alive until the copy has been consumed
            # the consumer's stream must not reuse the device blob before its own work is done
            b._blob.record_stream(cur)
        return b

    def close(self):
        """Stop the feeder thread (it finishes the batch in hand) and wait for it."""
        self._stop = True
        while self._th.is_alive():
            try:
                self._q.get(timeout=0.1)
            except queue.Empty:
                pass
        self._th.join()
