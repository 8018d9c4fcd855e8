#!/bin/bash
# GPU box: head tests, then c2 bench A/B of the in-tree build vs lib_base (AIMX_LIB_PATH),
# interleaved twice, then the GEMM tile-shape A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hab
B=aimnet-x2d_amd/lib_base/libaimx.so
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "head" > gpurun_out/hab/tests.log 2>&1 || { tail -20 gpurun_out/hab/tests.log; exit 1; }
tail -1 gpurun_out/hab/tests.log
for i in 1 2; do
  for v in base new; do
    ev=""; [ $v = base ] && ev="AIMX_LIB_PATH=$B"
    timeout -k 10 200 env $ev python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 40 > gpurun_out/hab/c2_${v}_$i.log 2>&1 || exit 1
    echo "c2 $v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hab/c2_${v}_$i.log)"
  done
done
tools/gpu_tile_ab.sh
