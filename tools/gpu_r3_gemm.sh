#!/bin/bash
# Round 3: 160-wide GEMM tiles and 160-wide weight-gradient blocks: parity, then step A/Bs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_gemm; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "wgrad or adam or gemm" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in c4 c5; do
  for bb in 80 160; do
    AIMX_WGRAD_BB=$bb timeout -k 10 120 python -u tools/wgrad_micro.py $c 0,256,1024 >> $O/micro.txt 2>&1 || { echo micro failed; tail $O/micro.txt; exit 1; }
    echo "bb=$bb $(tail -1 $O/micro.txt)"
  done
done
for c in c2 c4 c5; do
  for env in "AIMX_WGRAD_BB=80" "AIMX_WGRAD_BB=0" "AIMX_GEMM_WIDE=32" "AIMX_GEMM_WIDE=64"; do
    env $env timeout -k 10 300 python -u bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-roofline \
      --no-eager > $O/bench.json 2> $O/bench.err || { echo "bench $c $env failed"; tail -20 $O/bench.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" $O/bench.json $c "$env" | tee -a $O/ab.txt
  done
done
