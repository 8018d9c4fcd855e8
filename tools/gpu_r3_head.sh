#!/bin/bash
# Round 3: the fused head at F = 512 (c4): parity vs the module path, then step A/Bs over the
# width limit and the cluster size; c2 unchanged check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_head; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "head" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for env in "AIMX_HEAD_MAX_F=256" "AIMX_HEAD_CLUSTER=1" "AIMX_HEAD_CLUSTER=2" "AIMX_HEAD_CLUSTER=4" "AIMX_HEAD_CLUSTER=8"; do
  env $env timeout -k 10 300 python -u bench.py --config c4 --steps 50 --warmup 10 --no-cpu-baseline --no-roofline \
    --no-eager > $O/bench.json 2> $O/bench.err || { echo "bench c4 $env failed"; tail -20 $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" $O/bench.json c4 "$env" | tee -a $O/ab.txt
done
for env in "AIMX_HEAD_MAX_F=256" "AIMX_HEAD_MAX_F=512"; do
  env $env timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline \
    --no-eager > $O/bench.json 2> $O/bench.err || { echo "bench c2 $env failed"; tail -20 $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" $O/bench.json c2 "$env" | tee -a $O/ab.txt
done
