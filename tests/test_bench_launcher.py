"""bench.py's own rank launcher (`python bench.py --gpus N` without torchrun): the environment each
rank gets, exit-code propagation, and the --gpus / WORLD_SIZE consistency check. CPU only: the
launched programs here are tiny scripts, never the GPU bench."""
import json
import os
import subprocess
import sys
import time

import pytest

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
