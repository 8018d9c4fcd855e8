"""HDF5 molecule stream: the reference's precomputed dataset files, read and written natively.

Reference:
  * writer  src/datasets/features.py:381-431, 537-596 precompute_and_write_hdf5_parallel_chunked:
            /data = vlen-uint8 pickled {'smiles', 'target', 'precomputed'} per molecule,
            /index_map int32, /metadata attrs (num_samples, task_type, max_hops,
            preprocessing_applied, estimated_valid_pct; sae group)
  * reader  src/datasets/molecular.py:102-329 HDF5MolecularIterableDataset (shuffle with a
            rank-seeded RNG, contiguous rank shards, skip None records)

Here the file I/O and the record decoding run in C++ (libaimx_h5.so over the HDF5 C library, with
a non-executing pickle decoder, include/aimx_h5.h) and land in a native molecule store that the
C++ collator batches (aimx.feed). `HDF5MolecularStream` mirrors the reference dataset's
constructor and iteration order; one deliberate fix: rank shards all have ceil(n / world)
records (the tail wraps to the start, as torch's DistributedSampler pads), where the reference's
contiguous split (molecular.py:228-237) leaves the last ranks short or empty and DDP then waits on
a rank that has run out of batches.
"""
from __future__ import annotations

import ctypes
import math
import os
import pickle
import queue
import random
import threading

import numpy as np

from . import feed as afeed

_HERE = os.path.dirname(os.path.abspath(__file__))
H5_LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libaimx_h5.so")
# the HDF5 C library h5py links; loaded by path first so libaimx_h5.so's DT_NEEDED resolves to it
HDF5_CANDIDATES = (os.environ.get("AIMX_HDF5_LIB", ""), "/opt/conda/lib/libhdf5.so.103")

c_i64, c_i32, c_ptr = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
_ERR = {-1: "invalid argument", -3: "out of host memory", -10: "HDF5 I/O error", -11: "not the reference layout"}


class H5Info(ctypes.Structure):
    _fields_ = [("n_records", c_i64), ("num_samples", c_i64), ("max_hops", c_i64),
                ("preprocessing_applied", c_i32), ("task_type", ctypes.c_char * 32), ("direct_read", c_i32)]


_lib = None


def load_h5():
    """Load libaimx_h5.so (and the HDF5 C library it links); raises HostError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    afeed.load_host()
    for cand in HDF5_CANDIDATES:
        if cand and os.path.exists(cand):
            ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            break
    if not os.path.exists(H5_LIB_PATH):
        raise afeed.HostError(f"{H5_LIB_PATH} not built (run make -C aimnet-x2d_amd/csrc)")
    lib = ctypes.CDLL(H5_LIB_PATH)
    P = ctypes.POINTER
    lib.aimx_h5_open.restype = c_i32
    lib.aimx_h5_open.argtypes = [ctypes.c_char_p, P(c_ptr)]
    lib.aimx_h5_close.argtypes = [c_ptr]
    lib.aimx_h5_set_direct.restype = None
    lib.aimx_h5_set_direct.argtypes = [c_i32]
    lib.aimx_h5_info.restype = c_i32
    lib.aimx_h5_info.argtypes = [c_ptr, P(H5Info)]
    lib.aimx_h5_read_store.restype = c_i32
    lib.aimx_h5_read_store.argtypes = [c_ptr, c_ptr, c_i64, c_i32, c_i32, c_i32, P(c_ptr), P(c_i64), c_ptr]
    lib.aimx_h5_writer_create.restype = c_i32
    lib.aimx_h5_writer_create.argtypes = [ctypes.c_char_p, c_i64, P(H5Info), P(c_ptr)]
    lib.aimx_h5_writer_put.restype = c_i32
    lib.aimx_h5_writer_put.argtypes = [c_ptr, c_i64, c_i64, c_ptr, c_ptr]
    lib.aimx_h5_writer_close.restype = c_i32
    lib.aimx_h5_writer_close.argtypes = [c_ptr, ctypes.c_double]
    lib.aimx_h5_decode_record.restype = c_i32
    lib.aimx_h5_decode_record.argtypes = [c_ptr, c_i64, c_i32, c_i32, P(c_i32), P(c_i64)]
    _lib = lib
    return lib


def _check(rc, what):
    if rc < 0:
        raise afeed.HostError(f"aimx_h5 {what}: {_ERR.get(int(rc), rc)}")
    return rc


# ------------------------------------------------------------------------------------------- write
def make_record(n_atoms, bonds, feats, max_hops, target, total_charge=0, smiles=""):
    """One molecule in the reference's record layout (features.py:318-334, 556-561): BFS hop
    arrays int32 [2, E_h] (max_hops of them, empty ones included), atom features int8 columns,
    no stereo tensors, atomic numbers int32."""
    hops = afeed.bfs_multi_hop(int(n_atoms), bonds, max_hops)
    feats = np.asarray(feats).reshape(int(n_atoms), -1)
    af = {k: feats[:, i].astype(np.int8) for i, k in enumerate(afeed.adata.FEATURE_KEYS)}
    return {"smiles": smiles, "target": target, "precomputed": {
        "multi_hop_edges": [np.ascontiguousarray(h, np.int32).reshape(2, -1) for h in hops],
        "atom_features": af, "chiral_tensors": [], "cis_bonds_tensors": [], "trans_bonds_tensors": [],
        "total_charge": total_charge, "atomic_numbers": feats[:, 0].astype(np.int32) + 1,
        "processed_smiles": smiles}}


def write_hdf5(path, records, max_hops, task_type="regression", preprocessing_applied=True, chunk_size=1000):
    """precompute_and_write_hdf5_parallel_chunked's file from already-built records (dicts, or None
    for an invalid molecule): each is pickle.dumps'd exactly as features.py:551-561 does and written
    in chunks (a `bytes` item is taken as an already-pickled record). Returns the count."""
    lib = load_h5()
    records = list(records) if not hasattr(records, "__len__") else records
    n = len(records)
    info = H5Info(n, n, max_hops, int(bool(preprocessing_applied)), task_type.encode()[:31])
    w = c_ptr()
    _check(lib.aimx_h5_writer_create(os.fsencode(path), n, ctypes.byref(info), ctypes.byref(w)), "writer_create")
    valid = 0
    try:
        it = iter(records)
        for start in range(0, n, chunk_size):
            blobs = []
            for _ in range(min(chunk_size, n - start)):
                r = next(it)
                if isinstance(r, (bytes, bytearray)):  # an already-pickled record (parallel producers)
                    valid += 1
                    blobs.append(bytes(r))
                    continue
                valid += r is not None and r.get("precomputed") is not None
                blobs.append(pickle.dumps(r))
            offs = np.zeros(len(blobs) + 1, np.int64)
            offs[1:] = np.cumsum([len(b) for b in blobs])
            buf = np.frombuffer(b"".join(blobs), np.uint8)
            _check(lib.aimx_h5_writer_put(w, start, len(blobs), buf.ctypes.data if buf.size else None,
                                          offs.ctypes.data), "writer_put")
    finally:
        _check(lib.aimx_h5_writer_close(w, 100.0 * valid / max(n, 1)), "writer_close")
    return n


def decode_record(blob, n_hops, n_tasks=1):
    """C++ decoder on one pickled record: (valid, n_atoms, n_pairs)."""
    lib = load_h5()
    b = np.frombuffer(blob, np.uint8)
    na, npairs = c_i32(), c_i64()
    rc = _check(lib.aimx_h5_decode_record(b.ctypes.data if b.size else None, b.size, n_hops, n_tasks,
                                          ctypes.byref(na), ctypes.byref(npairs)), "decode_record")
    return bool(rc), int(na.value), int(npairs.value)


# -------------------------------------------------------------------------------------------- read
class H5File:
    """An open stream file (reader handle)."""

    def __init__(self, path):
        self._lib = load_h5()
        h = c_ptr()
        _check(self._lib.aimx_h5_open(os.fsencode(path), ctypes.byref(h)), f"open {path}")
        self._h = h
        info = H5Info()
        _check(self._lib.aimx_h5_info(h, ctypes.byref(info)), "info")
        self.n_records = int(info.n_records)
        self.num_samples = int(info.num_samples)
        self.max_hops = int(info.max_hops)
        self.preprocessing_applied = bool(info.preprocessing_applied)
        self.task_type = info.task_type.decode()
        self.direct_read = bool(info.direct_read)
        self._mtx = threading.Lock()  # one read at a time per handle

    def read_store(self, positions, n_hops, n_tasks=1, threads=4):
        """Records index_map[positions] -> (HostStore of the valid ones, positions kept)."""
        pos = np.ascontiguousarray(positions, np.int64)
        out, nv = c_ptr(), c_i64()
        kept = np.empty(max(pos.size, 1), np.int64)
        with self._mtx:
            _check(self._lib.aimx_h5_read_store(self._h, pos.ctypes.data if pos.size else None, pos.size, n_hops,
                                                n_tasks, threads, ctypes.byref(out), ctypes.byref(nv),
                                                kept.ctypes.data), "read_store")
            info = H5Info()
            if self._lib.aimx_h5_info(self._h, ctypes.byref(info)) == 0:
                self.direct_read = bool(info.direct_read)  # off once the file changed since open
        store = afeed.HostStore.from_handle(out, n_feat=len(afeed.adata.FEATURE_KEYS), n_tasks=n_tasks)
        return store, kept[:nv.value].copy()

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.aimx_h5_close(h)
            self._h = None

    def __del__(self):
        self.close()


def rank_shard(indices, rank, world_size):
    """Equal shards: every rank gets ceil(n / world) indices, contiguous in `indices`, the tail
    wrapping to the start (reference molecular.py:228-237 splits into ceil-size chunks and leaves
    the last ranks short)."""
    n = len(indices)
    if n == 0:
        return list(indices)
    per = int(math.ceil(n / float(world_size)))
    start = rank * per
    return [indices[(start + k) % n] for k in range(per)]


class HDF5MolecularStream:
    """Native counterpart of HDF5MolecularIterableDataset (molecular.py:102-329): same constructor
    arguments, same shuffle (random.Random seeded from torch.initial_seed() + seed + 10000 * rank
    when shuffle is on) and index_map; yields molecule stores instead of per-molecule Data
    objects. `chunks(chunk_size)` prefetches the next chunk on a background thread."""

    def __init__(self, hdf5_path, shuffle=False, buffer_size=1000, ddp_enabled=False, rank=0, world_size=1,
                 fold_indices=None, cv_fold=None, seed=42, n_hops=None, n_tasks=1, threads=4):
        self.file = H5File(hdf5_path)
        self.hdf5_path = hdf5_path
        self.shuffle, self.buffer_size, self.seed = shuffle, buffer_size, seed
        self.ddp_enabled, self.rank, self.world_size = ddp_enabled, rank, world_size
        self.fold_indices = fold_indices
        self.cv_fold = cv_fold
        self.n_hops = int(n_hops if n_hops is not None else max(self.file.max_hops, 1))
        self.n_tasks = int(n_tasks)
        self.threads = threads
        self.data_is_preprocessed = self.file.preprocessing_applied

    def __len__(self):
        total = len(self.fold_indices) if self.fold_indices is not None else self.file.n_records
        return int(math.ceil(total / float(self.world_size))) if self.ddp_enabled else total

    def positions(self, epoch_seed=None):
        """This rank's record positions for one pass (molecular.py:194-237, equal shards)."""
        idx = list(self.fold_indices) if self.fold_indices is not None else list(range(self.file.n_records))
        if self.shuffle:
            if epoch_seed is None:
                import torch
                epoch_seed = torch.initial_seed()
            rng = random.Random((epoch_seed + self.seed + self.rank * 10000) % (2 ** 32 - 1))
            rng.shuffle(idx)
        if self.ddp_enabled:
            idx = rank_shard(idx, self.rank, self.world_size)
        return np.asarray(idx, np.int64)

    def chunks(self, chunk_size=65536, epoch_seed=None, prefetch=2):
        """Yield (HostStore, kept positions) per chunk of this rank's positions; the next chunks are
        read and decoded on a background thread while the current one is consumed."""
        pos = self.positions(epoch_seed)
        q = queue.Queue(maxsize=max(1, prefetch))
        stop = threading.Event()

        def run():
            try:
                for s in range(0, len(pos), chunk_size):
                    if stop.is_set():
                        break
                    q.put(self.file.read_store(pos[s:s + chunk_size], self.n_hops, self.n_tasks, self.threads))
            except Exception as e:  # surfaced to the consumer
                q.put(e)
            q.put(None)

        th = threading.Thread(target=run, daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, Exception):
                    raise item
                yield item
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get(timeout=0.05)
                except queue.Empty:
                    pass

    def batches(self, batch_size, chunk_size=65536, epoch_seed=None, drop_last=True):
        """(store, molecule-index array) pairs for aimx.feed.BatchFeeder: batches never span chunks."""
        for store, _ in self.chunks(chunk_size, epoch_seed):
            n = len(store)
            stop = n - n % batch_size if drop_last else n
            for s in range(0, stop, batch_size):
                yield store, np.arange(s, min(s + batch_size, n), dtype=np.int64)


# ----------------------------------------------------------------------------- synthetic streams
def _synth_chunk(args):
    """Worker: pickled records [lo, hi) of a synthetic stream (deterministic per molecule index)."""
    lo, hi, source, hops, tasks, seed = args
    from .synth import QM9Asset, synth_molecule
    out = []
    asset = QM9Asset() if source == "qm9" else None
    for k in range(lo, hi):
        rng = np.random.default_rng([seed, k])
        if asset is not None:
            n, bonds, feats = asset.molecule(int(rng.integers(0, len(asset))))
        else:
            n, bonds, feats = synth_molecule(rng)
        target = float(rng.standard_normal()) if tasks == 1 else rng.standard_normal(tasks).astype(float).tolist()
        out.append(pickle.dumps(make_record(n, bonds, feats, hops, target, 0, f"syn{k}")))
    return out


def make_synthetic_stream(path, n_mols, source="synth40", hops=3, tasks=1, seed=0, workers=8, chunk=2048):
    """A synthetic stream file in the reference format: `source` 'synth40' (aimx.synth 40-atom
    molecules) or 'qm9' (QM9-val graphs resampled). Records are built and pickled by
    `workers` processes and written in order by this one."""
    import multiprocessing as mp
    jobs = [(lo, min(lo + chunk, n_mols), source, hops, tasks, seed) for lo in range(0, n_mols, chunk)]

    def records(pool):
        for blobs in pool.imap(_synth_chunk, jobs):
            yield from blobs

    class _Sized:
        def __init__(self, it):
            self.it = it

        def __len__(self):
            return n_mols

        def __iter__(self):
            return self.it

    ctx = mp.get_context("fork")
    with ctx.Pool(max(1, workers)) as pool:
        return write_hdf5(path, _Sized(records(pool)), hops, task_type="regression" if tasks == 1 else "multitask",
                          chunk_size=chunk)
