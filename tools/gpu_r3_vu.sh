#!/bin/bash
# Round 3: 16-byte staging of unaligned k-contiguous GEMM operands (k_gemm VU): parity, A/B steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_vu; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "gemm or wgrad or layer or model or mlp" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in c4 c5 c3; do
  for env in "AIMX_GEMM_VU=0" "AIMX_GEMM_VU=1"; do
    env $env timeout -k 10 300 python -u bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-roofline \
      --no-eager > $O/bench.json 2> $O/bench.err || { echo "bench $c $env failed"; tail -20 $O/bench.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" $O/bench.json $c "$env" | tee -a $O/ab.txt
  done
done
