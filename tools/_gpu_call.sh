#!/bin/bash
# round-6 working call (overwritten per call): full -m gpu suite after the knob pruning + the
# large-tile GEMM, then the big-GEMM variants (tuning build) and c2 / c5 bench lines
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python3 -u -m pytest -x -q --timeout 200 --timeout-method thread"
TL=aimnet-x2d_amd/lib/libaimx_tune.so
tools/gpu_steps.sh \
  "300 r6c/gemm_old.log AIMX_LIB_PATH=$TL AIMX_GEMM_BIG=0 python3 tools/gemm_micro.py big" \
 "300 r6c/gemm_w8.log AIMX_LIB_PATH=$TL AIMX_GEMM_BIG_W=8 python3 tools/gemm_micro.py big" \
 "300 r6c/gemm_w4.log AIMX_LIB_PATH=$TL AIMX_GEMM_BIG_W=4 python3 tools/gemm_micro.py big" \
 "300 r6c/gemm_w8_128.log AIMX_LIB_PATH=$TL AIMX_GEMM_BIG_W=8 AIMX_GEMM_BIG=128 python3 tools/gemm_micro.py big" \
 "300 r6c/gemm_w8_64.log AIMX_LIB_PATH=$TL AIMX_GEMM_BIG_W=8 AIMX_GEMM_BIG=64 python3 tools/gemm_micro.py big" \
 "300 r6c/c5.log python3 bench.py --config c5 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6c/c5_old.log AIMX_LIB_PATH=$TL AIMX_GEMM_BIG=0 python3 bench.py --config c5 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6c/c4.log python3 bench.py --config c4 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6c/c2.log python3 bench.py --no-cpu-baseline --no-eager --no-roofline" \
 "900 r6c/tests.log python3 -u -m pytest -q --maxfail 5 --timeout 200 --timeout-method thread tests -m gpu"
