#!/bin/bash
# Round 3: software-pipelined LDS fragment reads (k_wgrad_lds, k_gemm): parity, micro and step A/B
# against a variant library built with -DAIMX_LDS_PIPE=0 (aimnet-x2d_amd/lib_nopipe).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_pipe; mkdir -p $O
NP=$PWD/aimnet-x2d_amd/lib_nopipe/libaimx.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_amp.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in c2 c4 c5; do
  for v in pipe nopipe; do
    if [ $v = nopipe ]; then export AIMX_LIB_PATH=$NP; else unset AIMX_LIB_PATH; fi
    timeout -k 10 120 python -u tools/wgrad_micro.py $c > $O/micro.txt 2>&1 || { echo micro failed; tail $O/micro.txt; exit 1; }
    echo "$v $(grep '^{' $O/micro.txt | tail -1)" | tee -a $O/ab.txt
    timeout -k 10 300 python -u bench.py --config $c --steps 60 --warmup 10 --no-cpu-baseline --no-roofline \
      --no-eager > $O/bench.json 2> $O/bench.err || { echo "bench $c $v failed"; tail -20 $O/bench.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" $O/bench.json $c $v | tee -a $O/ab.txt
  done
done
