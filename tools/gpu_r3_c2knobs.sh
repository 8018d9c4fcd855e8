#!/bin/bash
# Round 3: grouped weight-gradient K per workgroup (group rule) and the c2 head cluster size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_c2knobs; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py \
  -k "wgrad or adam or gemm_ones or full_train or head" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python -u tools/wgrad_micro.py c2 0,512 > $O/micro.txt 2>&1 || { echo micro failed; tail $O/micro.txt; exit 1; }
cat $O/micro.txt
run() {  # name env... -- config
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config $CFG --steps 100 --warmup 10 --no-cpu-baseline --no-roofline \
    --no-eager > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $name failed"; tail -20 $O/bench_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" $O/bench_$name.json $name
}
CFG=c2
run c2_default AIMX_X=0
run c2_kper512 AIMX_WGRAD_KPER=512
run c2_cluster4 AIMX_HEAD_CLUSTER=4
run c2_cluster8 AIMX_HEAD_CLUSTER=8
run c2_default2 AIMX_X=0
CFG=c4
run c4_default AIMX_X=0
CFG=c5
run c5_default AIMX_X=0
