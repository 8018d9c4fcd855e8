#!/bin/bash
# round-6 working call (overwritten per call): atoms per k_wgrad_lds workgroup (AIMX_WGRAD_KPER,
# tuning build): the grouped micro at the stack's 16-byte rows, then c5 / c4 / c2 steps
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TL=aimnet-x2d_amd/lib/libaimx_tune.so
B="python3 bench.py --no-cpu-baseline --no-eager --no-roofline"
tools/gpu_steps.sh \
 "200 r6k/m_c5.log AIMX_LIB_PATH=$TL python3 tools/wgrad_micro.py c5 0,1024,2048" \
 "200 r6k/m_c4.log AIMX_LIB_PATH=$TL python3 tools/wgrad_micro.py c4 0,1024,2048" \
 "300 r6k/c5_512.log AIMX_LIB_PATH=$TL $B --config c5" \
 "300 r6k/c5_1024.log AIMX_LIB_PATH=$TL AIMX_WGRAD_KPER=1024 $B --config c5" \
 "300 r6k/c5_2048.log AIMX_LIB_PATH=$TL AIMX_WGRAD_KPER=2048 $B --config c5" \
 "300 r6k/c4_512.log AIMX_LIB_PATH=$TL $B --config c4" \
 "300 r6k/c4_1024.log AIMX_LIB_PATH=$TL AIMX_WGRAD_KPER=1024 $B --config c4" \
 "300 r6k/c2_512.log AIMX_LIB_PATH=$TL $B" \
 "300 r6k/c2_256.log AIMX_LIB_PATH=$TL AIMX_WGRAD_KPER=256 $B"
