#!/bin/bash
# GPU box: GEMM tile-shape A/B (AIMX_GEMM_TILE) on the graph-timed hot-path shapes and the c2 step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tile
for t in default 64x32 32x32; do
  ev=""; [ "$t" != "default" ] && ev="AIMX_GEMM_TILE=$t"
  timeout -k 10 200 env $ev python3 tools/gemm_micro.py > gpurun_out/tile/gemm_$t.log 2>&1 || exit 1
  timeout -k 10 200 env $ev python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 40 > gpurun_out/tile/c2_$t.log 2>&1 || exit 1
  echo "$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tile/c2_$t.log)"
done
