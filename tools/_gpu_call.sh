#!/bin/bash
# round-6 working call (overwritten per call): the c5 1 M-molecule stream line + feed rate (profile
# part s), then the deep GEMM's round-robin k variant (tuning build) against the default
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TL=aimnet-x2d_amd/lib/libaimx_tune.so
bash tools/profile_round.sh s && tools/gpu_steps.sh \
 "200 r6i/deep16.log AIMX_LIB_PATH=$TL python3 tools/gemm_micro.py deep" \
 "200 r6i/deep16_il.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP_IL=1 python3 tools/gemm_micro.py deep" \
 "200 r6i/deep8_il.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP_IL=1 AIMX_GEMM_DEEP=8 python3 tools/gemm_micro.py deep"
