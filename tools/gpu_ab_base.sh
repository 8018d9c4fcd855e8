#!/bin/bash
# GPU box: full -m gpu suite on the in-tree build, then bench A/B (in-tree vs lib_base via
# AIMX_LIB_PATH) interleaved twice per config. usage: tools/gpu_ab_base.sh c2,c4
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abb
B=aimnet-x2d_amd/lib_base/libaimx.so
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/abb/tests.log 2>&1 || { tail -30 gpurun_out/abb/tests.log; exit 1; }
tail -1 gpurun_out/abb/tests.log
for c in ${1//,/ }; do
  for i in 1 2; do
    for v in base new; do
      ev=""; [ $v = base ] && ev="AIMX_LIB_PATH=$B"
      timeout -k 10 200 env $ev python3 bench.py --config $c --no-cpu-baseline --no-roofline --no-eager --steps 40 > gpurun_out/abb/${c}_${v}_$i.log 2>&1 || exit 1
      echo "$c $v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abb/${c}_${v}_$i.log)"
    done
  done
done
