#!/bin/bash
# Round 3: double-buffered LDS in k_wgrad_lds (AIMX_WGRAD_DBUF): parity, micro A/B, steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_dbuf; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py \
  -k "wgrad or adam or gemm_ones or full_train" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in c2 c4 c5; do
  for db in 0 1; do
    AIMX_WGRAD_DBUF=$db timeout -k 10 120 python -u tools/wgrad_micro.py $c 0,256,1024 >> $O/micro.txt 2>&1 || { echo micro failed; tail $O/micro.txt; exit 1; }
    echo "dbuf=$db $(tail -1 $O/micro.txt)"
  done
done
for c in c2 c4 c5; do
  for db in 0 1; do
    AIMX_WGRAD_DBUF=$db timeout -k 10 300 python -u bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-roofline \
      --no-eager > $O/bench_${c}_$db.json 2> $O/bench_${c}_$db.err || { echo "bench $c failed"; tail -20 $O/bench_${c}_$db.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/bench_${c}_$db.json
  done
done
