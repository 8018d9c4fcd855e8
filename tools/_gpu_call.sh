#!/bin/bash
# round-6 working call (overwritten per call): k_gemm_deep as 16x16x4 sub-tiles (AIMX_GEMM_DEEP_M16,
# tuning build): parity tests on it, the micro, c5 / c4 steps against the 32x32x2 default
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TL=aimnet-x2d_amd/lib/libaimx_tune.so
A="--no-cpu-baseline --no-eager --no-roofline"
tools/gpu_steps.sh \
 "300 r6n/tests_m16.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP_M16=1 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'deep or head_path or few_rows'" \
 "200 r6n/m32.log AIMX_LIB_PATH=$TL python3 tools/gemm_micro.py deep" \
 "200 r6n/m16.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP_M16=1 python3 tools/gemm_micro.py deep" \
 "300 r6n/c5_32.log AIMX_LIB_PATH=$TL python3 bench.py --config c5 $A" \
 "300 r6n/c5_16.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP_M16=1 python3 bench.py --config c5 $A" \
 "300 r6n/c4_32.log AIMX_LIB_PATH=$TL python3 bench.py --config c4 $A" \
 "300 r6n/c4_16.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP_M16=1 python3 bench.py --config c4 $A"
