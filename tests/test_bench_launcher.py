"""bench.py's own rank launcher (`python bench.py --gpus N` without torchrun): the environment each
rank gets, exit-code propagation, and the --gpus / WORLD_SIZE consistency check. CPU only: the
launched programs here are tiny scripts, never the GPU bench."""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_rank_env_is_torchrun_compatible():
    base = {"PATH": "/usr/bin", "WORLD_SIZE_UNRELATED": "x"}
    envs = [bench.rank_env(base, r, 8, 29555) for r in range(8)]
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "8"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert e["PATH"] == "/usr/bin"
    assert "RANK" not in base  # the caller's environment is not modified
    # an explicit setting in the parent environment wins
    assert bench.rank_env({"HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 0, 2, 1)["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text("import json, os, sys, time\n" + body)
    return str(p)


def test_launch_ranks_starts_n_ranks_and_relays_rank0(tmp_path, capfd):
    out = tmp_path / "seen"
    out.mkdir()
    script = _script(tmp_path, f"""
r = int(os.environ["RANK"])
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
open(os.path.join({str(out)!r}, str(r)), "w").write(json.dumps({{k: os.environ[k] for k in keys}}))
if r == 0:
    print(json.dumps({{"rank0_line": sys.argv[1:]}}))
else:
    print("not the line")
""")
    rc = bench.launch_ranks(3, ["--gpus", "3"], script=script)
    assert rc == 0
    seen = {int(f): json.loads((out / f).read_text()) for f in os.listdir(out)}
    assert sorted(seen) == [0, 1, 2]
    assert len({s["MASTER_PORT"] for s in seen.values()}) == 1
    assert all(s["WORLD_SIZE"] == "3" and s["LOCAL_RANK"] == s["RANK"] for s in seen.values())
    o, e = capfd.readouterr()
    assert o.strip().splitlines() == ['{"rank0_line": ["--gpus", "3"]}']  # rank 0 only on stdout
    assert "not the line" in e


def test_launch_ranks_failure_stops_peers(tmp_path):
    script = _script(tmp_path, """
if os.environ["RANK"] == "1":
    sys.exit(7)
time.sleep(120)  # a peer stuck in a collective
""")
    t0 = time.time()
    rc = bench.launch_ranks(2, [], script=script)
    assert rc == 7
    assert time.time() - t0 < 60


def test_launch_ranks_signal_exit_code(tmp_path):
    script = _script(tmp_path, "import signal\nif os.environ['RANK'] == '0':\n    os.kill(os.getpid(), signal.SIGKILL)\n")
    assert bench.launch_ranks(2, [], script=script) == 128 + 9


@pytest.mark.parametrize("world,gpus", [("1", "2"), ("4", "8"), ("2", "1")])
def test_gpus_must_equal_world_size(world, gpus):
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", gpus], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr
    assert f"--gpus {gpus} but WORLD_SIZE {world}" in p.stderr
    assert p.stdout == ""


def _alive(pid):
    """True while pid exists and is not a zombie."""
    try:
        with open(f"/proc/{pid}/status") as f:
            return not any(ln.startswith("State:") and "Z" in ln.split()[1] for ln in f)
    except FileNotFoundError:
        return False


def _launcher(tmp_path, n, body, extra=""):
    """A separate launcher process (python -> bench.launch_ranks) whose ranks write their pids."""
    pids = tmp_path / "pids"
    pids.mkdir()
    script = _script(tmp_path, f"open(os.path.join({str(pids)!r}, os.environ['RANK']), 'w').write(str(os.getpid()))\n"
                     + body)
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.launch_ranks({n}, [], script={script!r}{extra}))")
    p = subprocess.Popen([sys.executable, "-c", code], start_new_session=True)
    t0 = time.time()
    while len(os.listdir(pids)) < n and time.time() - t0 < 120:
        time.sleep(0.05)
    assert len(os.listdir(pids)) == n, "ranks did not start"
    return p, [int((pids / f).read_text()) for f in sorted(os.listdir(pids))]


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGHUP", "SIGINT"])
def test_launcher_signal_stops_every_rank(tmp_path, sig):
    """The driver's timeout signals the launcher: every rank is gone within 5 s and the launcher
    exits 128 + the signal."""
    import signal
    p, pids = _launcher(tmp_path, 3, "time.sleep(300)\n")
    p.send_signal(getattr(signal, sig))
    assert p.wait(timeout=30) == 128 + int(getattr(signal, sig))
    t0 = time.time()
    while any(_alive(q) for q in pids) and time.time() - t0 < 5:
        time.sleep(0.05)
    assert not any(_alive(q) for q in pids)


def test_launcher_killed_outright_takes_its_ranks(tmp_path):
    """SIGKILL cannot be forwarded: the ranks' parent-death signal ends them within 5 s."""
    import signal
    p, pids = _launcher(tmp_path, 2, "time.sleep(300)\n")
    p.send_signal(signal.SIGKILL)
    p.wait(timeout=30)
    t0 = time.time()
    while any(_alive(q) for q in pids) and time.time() - t0 < 5:
        time.sleep(0.05)
    assert not any(_alive(q) for q in pids)


def test_hung_rank_with_finished_peer_hits_the_deadline(tmp_path):
    """Rank 0 finishes, rank 1 hangs (a collective that never completes): the launcher stops it
    and exits non-zero by the deadline (and by the straggler window, whichever comes first)."""
    body = "if os.environ['RANK'] == '1':\n    time.sleep(300)\n"
    for extra, limit in ((", deadline_s=3.0", 20), (", straggler_s=2.0", 20)):
        sub = tmp_path / extra.strip(", =.").replace("=", "")
        sub.mkdir()
        t0 = time.time()
        p, pids = _launcher(sub, 2, body, extra)
        assert p.wait(timeout=60) == 124
        assert time.time() - t0 < limit
        t1 = time.time()
        while any(_alive(q) for q in pids) and time.time() - t1 < 5:
            time.sleep(0.05)
        assert not any(_alive(q) for q in pids)


@pytest.mark.parametrize("config,buckets", [("c2", True), ("c5", True), ("c4", False)])
def test_padded_static_layouts_on_cpu(config, buckets):
    """bench.make_batches' static graph layouts (the default bench path): every batch padded to its
    bucket's atom count (a multiple of the config's layout quantum), padding molecules appended and
    excluded from the loss by real_graphs, charges and targets padded with zeros."""
    cfg = dict(bench.CONFIGS[config])
    cfg["batch"] = 12
    q = bench.layout_quantum(cfg)
    bs = bench.make_batches(cfg, 3, 7, torch.device("cpu"), pad=True, buckets=buckets)
    assert len(bs) == 3
    for b in bs:
        n = b.batch.shape[0]
        if buckets:
            assert n % q == 0 and n >= b.real_atoms + 2
        assert b.real_graphs == 12 and b.total_charges.shape[0] > 12
        assert not b.total_charges[12:].any()


def test_multi_gpu_runs_get_a_default_deadline():
    assert bench.resolve_deadline(1, None) == 0.0
    assert bench.resolve_deadline(8, None) == bench.DEFAULT_DEADLINE_S > 0
    assert bench.resolve_deadline(8, 0) == 0.0 and bench.resolve_deadline(2, 45) == 45.0


def test_rank_watchdog_ends_a_hung_rank(tmp_path):
    """A rank stuck in a collective (here: a sleep) exits 124 at its own deadline, so torchrun (or
    launch_ranks) sees a failure and stops its peers; a rank that finishes first exits normally."""
    hung = _script(tmp_path, f"sys.path.insert(0, {ROOT!r}); import bench; bench.rank_watchdog(1.0); time.sleep(60)\n")
    t0 = time.time()
    p = subprocess.run([sys.executable, hung], capture_output=True, text=True, timeout=60)
    assert p.returncode == 124 and time.time() - t0 < 30
    assert "deadline of 1 s passed" in p.stderr
    ok = tmp_path / "ok.py"
    ok.write_text(f"import sys; sys.path.insert(0, {ROOT!r}); import bench; bench.rank_watchdog(30.0); print('done')\n")
    p = subprocess.run([sys.executable, str(ok)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and p.stdout.strip() == "done"


def test_exit_codes_after_the_line(capsys):
    """Diverged replicas fail the command (3); an RCCL capture that fell back to split graphs is a
    valid split-mode measurement (0, with a warning) — the first 8-GPU driver run must yield a record."""
    assert bench.exit_code(None, None) == 0
    assert bench.exit_code({"replicas_identical": True}, None) == 0
    assert bench.exit_code({"replicas_identical": True}, RuntimeError("capture failed")) == 0
    assert "fell back to split graphs" in capsys.readouterr().err
    assert bench.exit_code({"replicas_identical": False}, None) == 3
    assert bench.exit_code({"replicas_identical": False}, RuntimeError("x")) == 3
