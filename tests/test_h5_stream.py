"""HDF5 molecule stream (libaimx_h5.so, aimx.h5) vs the reference dataset format, CPU only.

Pinned by the committed byte-level fixture tests/golden/stream_small.h5 (written by
tests/golden/make_stream_fixture.py with Python's pickle and the HDF5 C library) and its expected
collate (tests/golden/stream_small_expected.npz, the reference collate restated in pure Python on
pickle.loads of the same records): bit-exact. h5py itself is not installable here; the layout is
checked with the HDF5 tools' h5dump instead (the same library h5py links)."""
import os
import pickle
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from aimx import data as adata
from aimx import feed, h5
from aimx.synth import synth_molecules

FIX = os.path.join(ROOT, "tests", "golden", "stream_small.h5")
EXP = os.path.join(ROOT, "tests", "golden", "stream_small_expected.npz")


def _collate(store):
    return feed.HostCollator(3, threads=2).collate(store, np.arange(len(store)))


def test_fixture_reads_bit_exact():
    z = np.load(EXP)
    f = h5.H5File(FIX)
    assert f.n_records == 63 and f.max_hops == 3 and f.task_type == "regression" and f.preprocessing_applied
    store, kept = f.read_store(np.arange(f.n_records), 3, 1, threads=3)
    assert np.array_equal(kept, z["positions"])  # the two None records and the one without 'precomputed' skipped
    col = _collate(store)
    for k in ("edges", "feats", "batch", "n_atoms", "total_charges"):
        assert np.array_equal(col[k], z[k]), k
    assert np.array_equal(col["targets"][:, 0], z["targets"])


def test_fixture_random_access_and_order():
    """A point selection (non-contiguous, unsorted positions) returns records in request order."""
    z = np.load(EXP)
    f = h5.H5File(FIX)
    pos = np.array([40, 3, 3, 62, 0, 18], np.int64)
    store, kept = f.read_store(pos, 3, 1)
    assert np.array_equal(kept, pos)
    full, _ = f.read_store(np.arange(f.n_records), 3, 1)
    where = {int(p): i for i, p in enumerate(z["positions"])}
    col = _collate(store)
    ref = feed.HostCollator(3).collate(full, np.array([where[int(p)] for p in pos]))
    for k in ("edges", "feats", "batch", "n_atoms"):
        assert np.array_equal(col[k], ref[k]), k


@pytest.mark.skipif(not shutil.which("h5dump") and not os.path.exists("/opt/conda/bin/h5dump"),
                    reason="HDF5 tools absent")
def test_fixture_layout_is_h5py_layout():
    """The file h5py writes for features.py:416-431: vlen uint8 /data, int32 /index_map, int64
    attrs, bool as an int8 FALSE/TRUE enum, str as variable-length UTF-8."""
    exe = shutil.which("h5dump") or "/opt/conda/bin/h5dump"
    out = subprocess.run([exe, "-H", FIX], capture_output=True, text=True, check=True).stdout
    flat = " ".join(out.split())
    assert 'DATASET "data" { DATATYPE H5T_VLEN { H5T_STD_U8LE} DATASPACE SIMPLE { ( 63 ) / ( 63 ) }' in flat
    assert 'DATASET "index_map" { DATATYPE H5T_STD_I32LE' in flat
    assert 'ATTRIBUTE "num_samples" { DATATYPE H5T_STD_I64LE DATASPACE SCALAR' in flat
    assert 'ATTRIBUTE "preprocessing_applied" { DATATYPE H5T_ENUM { H5T_STD_I8LE; "FALSE" 0; "TRUE" 1; }' in flat
    assert 'ATTRIBUTE "task_type" { DATATYPE H5T_STRING { STRSIZE H5T_VARIABLE;' in flat
    assert 'GROUP "sae"' in flat


def test_writer_roundtrip(tmp_path):
    mols = synth_molecules(30, seed=5)
    recs = [h5.make_record(n, b, f, 4, [0.5 * i, -1.0 * i], total_charge=i % 2) for i, (n, b, f) in enumerate(mols)]
    p = str(tmp_path / "rt.h5")
    assert h5.write_hdf5(p, recs, 4, task_type="multitask", chunk_size=7) == 30
    f = h5.H5File(p)
    assert f.task_type == "multitask" and f.max_hops == 4
    store, kept = f.read_store(np.arange(30), 4, 2)
    assert len(store) == 30
    col = _collate_h(store, 4)
    ref = adata.collate([(n, b, np.asarray(fe, np.int64)) for n, b, fe in mols], 4)
    for k in ("edges", "feats", "batch", "n_atoms"):
        assert np.array_equal(col[k], ref[k]), k
    assert np.allclose(col["targets"], np.array([[0.5 * i, -1.0 * i] for i in range(30)], np.float32))
    # a 3-hop read of a 4-hop file takes the first three hop arrays
    s3, _ = f.read_store(np.arange(30), 3, 2)
    ref3 = adata.collate([(n, b, np.asarray(fe, np.int64)) for n, b, fe in mols], 3)
    assert np.array_equal(_collate_h(s3, 3)["edges"], ref3["edges"])


def _collate_h(store, hops):
    return feed.HostCollator(hops).collate(store, np.arange(len(store)))


def test_wrong_target_width_is_skipped(tmp_path):
    mols = synth_molecules(4, seed=1)
    recs = [h5.make_record(n, b, f, 3, 1.0) for n, b, f in mols]
    recs[2]["target"] = [1.0, 2.0]
    p = str(tmp_path / "w.h5")
    h5.write_hdf5(p, recs, 3)
    _, kept = h5.H5File(p).read_store(np.arange(4), 3, 1)
    assert kept.tolist() == [0, 1, 3]


class _Evil:
    def __reduce__(self):
        return (os.system, ("touch /tmp/aimx_pickle_pwned",))


def test_pickle_decoder_executes_nothing():
    """A record whose pickle names any global outside the numpy reconstructors is rejected,
    never called (the reference's pickle.loads would run it)."""
    if os.path.exists("/tmp/aimx_pickle_pwned"):
        os.remove("/tmp/aimx_pickle_pwned")
    mols = synth_molecules(1, seed=2)
    rec = h5.make_record(*mols[0], 3, 1.0)
    rec["precomputed"]["processed_smiles"] = _Evil()
    assert h5.decode_record(pickle.dumps(rec), 3) == (False, 0, 0)
    assert not os.path.exists("/tmp/aimx_pickle_pwned")
    ok, na, npairs = h5.decode_record(pickle.dumps(h5.make_record(*mols[0], 3, 1.0)), 3)
    assert ok and na == mols[0][0] and npairs > 0
    for proto in (2, 3, 5):  # other protocols the reference's Python may have used
        ok, na2, np2 = h5.decode_record(pickle.dumps(h5.make_record(*mols[0], 3, 1.0), protocol=proto), 3)
        assert ok and (na2, np2) == (na, npairs), proto
    assert h5.decode_record(b"\x80\x04garbage", 3)[0] is False


def test_malformed_array_shapes_are_rejected():
    """Protocol-5 records whose hop array claims a negative or oversized shape (2, -5) / (2, 2e9):
    the decoder rejects them (dims checked, numel * itemsize must equal the payload) instead of
    writing outside the record's buffer or throwing bad_alloc inside a worker thread."""
    import struct
    mols = synth_molecules(1, seed=3)
    rec = h5.make_record(*mols[0], 3, 1.0)
    e1 = rec["precomputed"]["multi_hop_edges"][0].shape[1]
    assert e1 < 256
    blob = pickle.dumps(rec, protocol=5)
    pat = b"K\x02K" + bytes([e1]) + b"\x86"  # the first hop array's shape tuple (2, E1)
    assert pat in blob
    assert h5.decode_record(blob, 3)[0] is True
    for bad in (-5, 2_000_000_000, 0x7FFFFFFF):
        evil = blob.replace(pat, b"K\x02J" + struct.pack("<i", bad) + b"\x86", 1)
        assert h5.decode_record(evil, 3) == (False, 0, 0), bad


def test_rank_shards_equal_and_covering():
    """Equal shard lengths (the reference's contiguous ceil split leaves the last ranks short or
    empty, molecular.py:228-237); every record appears; shuffle is seeded per rank."""
    for n, world in ((63, 4), (10, 3), (5, 8), (64, 8)):
        shards = [h5.rank_shard(list(range(n)), r, world) for r in range(world)]
        per = -(-n // world)
        assert all(len(s) == per for s in shards)
        assert set().union(*map(set, shards)) == set(range(n))
    s0 = h5.HDF5MolecularStream(FIX, shuffle=True, ddp_enabled=True, rank=1, world_size=4)
    assert len(s0) == 16
    a, b = s0.positions(epoch_seed=7), s0.positions(epoch_seed=7)
    assert np.array_equal(a, b) and len(a) == 16
    assert not np.array_equal(a, s0.positions(epoch_seed=8))


def test_stream_batches_span_chunks():
    """batches(): chunked reads (prefetched on a thread), each batch inside one chunk; together
    they cover the valid records in order."""
    z = np.load(EXP)
    s = h5.HDF5MolecularStream(FIX, n_hops=3)
    got = []
    for store, idx in s.batches(batch_size=8, chunk_size=20, drop_last=False):
        col = feed.HostCollator(3).collate(store, idx)
        got.append(col["n_atoms"])
    assert np.array_equal(np.concatenate(got), z["n_atoms"])


def _read_all(path, pos, hops, direct, threads=3):
    lib = h5.load_h5()
    lib.aimx_h5_set_direct(1 if direct else 0)  # test hook: the direct path allowed or not
    try:
        f = h5.H5File(path)
    finally:
        lib.aimx_h5_set_direct(1)
    assert f.direct_read == direct
    store, kept = f.read_store(pos, hops, 1, threads)
    return _collate_h(store, hops), kept


def test_direct_read_equals_hdf5_read(tmp_path):
    """The mapped-file path (records found in the global heap directly, no H5Dread) returns exactly
    what the HDF5 library returns: the fixture, and a file large enough that the open-time check
    samples only some records; unsorted positions with repeats (the H5Dread path sorts them)."""
    z = np.load(EXP)
    for path, n, hops in [(FIX, 63, 3), (None, 300, 3)]:
        if path is None:
            mols = synth_molecules(n, seed=9)
            recs = [h5.make_record(a, b, f, hops, 0.25 * i) for i, (a, b, f) in enumerate(mols)]
            recs[17] = None
            path = str(tmp_path / "big.h5")
            h5.write_hdf5(path, recs, hops, chunk_size=64)
        rng = np.random.default_rng(3)
        pos = np.concatenate([rng.permutation(n), rng.integers(0, n, 40)]).astype(np.int64)
        a, ka = _read_all(path, pos, hops, True)
        b, kb = _read_all(path, pos, hops, False)
        assert np.array_equal(ka, kb)
        for k in ("edges", "feats", "batch", "n_atoms", "total_charges", "targets"):
            assert np.array_equal(a[k], b[k]), k
        if path == FIX:
            full, kf = _read_all(FIX, np.arange(63), 3, True)
            assert np.array_equal(kf, z["positions"])
            assert np.array_equal(full["edges"], z["edges"])


def test_shuffled_read_equals_request_order(tmp_path):
    """Records are decoded in file order and placed in request order: a shuffled request with
    repeats and invalid records, on 1 / 3 / 8 threads and both read paths, collates exactly like
    the same molecules picked out of an in-order read."""
    n, hops = 120, 3
    mols = synth_molecules(n, seed=5)
    recs = [h5.make_record(a, b, f, hops, 0.5 * i, total_charge=i % 3 - 1) for i, (a, b, f) in enumerate(mols)]
    for bad in (7, 61, 119):
        recs[bad] = None
    path = str(tmp_path / "shuf.h5")
    h5.write_hdf5(path, recs, hops, chunk_size=32)
    rng = np.random.default_rng(11)
    pos = np.concatenate([rng.permutation(n), rng.integers(0, n, 30)]).astype(np.int64)
    want = [int(q) for q in pos if recs[int(q)] is not None]
    full, kf = h5.H5File(path).read_store(np.arange(n), hops, 1, 1)
    where = {int(q): i for i, q in enumerate(kf)}
    ref = feed.HostCollator(hops).collate(full, np.array([where[q] for q in want]))
    for direct in (True, False):
        for threads in (1, 3, 8):
            col, kept = _read_all(path, pos, hops, direct, threads=threads)
            assert kept.tolist() == want
            for k in ("edges", "feats", "batch", "n_atoms", "total_charges", "targets"):
                assert np.array_equal(col[k], ref[k]), (direct, threads, k)


def test_direct_read_never_returns_wrong_bytes(tmp_path):
    """A damaged global heap collection: the direct path is refused at open (sampled records
    differ from H5Dread's) or the read of a damaged record fails; it never yields other bytes."""
    mols = synth_molecules(200, seed=4)
    recs = [h5.make_record(a, b, f, 3, float(i)) for i, (a, b, f) in enumerate(mols)]
    good = str(tmp_path / "good.h5")
    h5.write_hdf5(good, recs, 3)
    raw = bytearray(open(good, "rb").read())
    hits = [i for i in range(len(raw) - 4) if raw[i:i + 4] == b"GCOL"]
    assert len(hits) >= 2
    ref, kref = _read_all(good, np.arange(200), 3, True)
    for victim in (hits[0], hits[len(hits) // 2]):
        bad = bytearray(raw)
        bad[victim + 3] = ord("X")
        p = str(tmp_path / f"bad{victim}.h5")
        open(p, "wb").write(bytes(bad))
        f = h5.H5File(p)
        if not f.direct_read:
            continue
        try:
            store, kept = f.read_store(np.arange(200), 3, 1, 3)
        except Exception:
            continue
        col = _collate_h(store, 3)
        assert np.array_equal(kept, kref) and np.array_equal(col["edges"], ref["edges"])


def test_file_changed_after_open_falls_back_from_the_mapping(tmp_path):
    """The direct path maps the file at open; a file modified afterwards (here: a copy of the
    fixture, its tail truncated away — a stream regenerated by another process) is no longer read
    through that mapping (which would fault past the new end): the reader re-checks the file's
    size and time before each read and drops to H5Dread, which fails with an error instead."""
    p = tmp_path / "s.h5"
    shutil.copy(FIX, p)
    f = h5.H5File(str(p))
    assert f.direct_read
    ok, _ = f.read_store(np.arange(f.n_records), 3, 1)
    assert len(ok) > 0
    os.truncate(p, os.path.getsize(p) // 2)
    try:
        f.read_store(np.arange(f.n_records), 3, 1)
    except Exception:  # H5Dread of the truncated file: an error, never a crash
        pass
    assert not f.direct_read
