#!/bin/bash
# GEMM A/B on the GPU box: GEMM parity tests on the in-tree build, then graph-timed GEMM shapes and
# the c2/c4 bench lines with the baseline build (lib_base/, AIMX_LIB_PATH) and the in-tree one.
set -o pipefail
export TMPDIR=/tmp
B=aimnet-x2d_amd/lib_base/libaimx.so
tools/gpu_steps.sh "300 gab/tests.log python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k gemm" \
  "300 gab/gemm_base.log env AIMX_LIB_PATH=$B python3 tools/gemm_micro.py" \
  "300 gab/gemm_new.log python3 tools/gemm_micro.py" \
  "300 gab/c2_base.log env AIMX_LIB_PATH=$B python3 bench.py --no-cpu-baseline --no-roofline --no-eager" \
  "300 gab/c2_new.log python3 bench.py --no-cpu-baseline --no-roofline --no-eager" \
  "300 gab/c4_base.log env AIMX_LIB_PATH=$B python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager" \
  "300 gab/c4_new.log python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager"
