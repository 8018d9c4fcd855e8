#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4p
B="python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline --no-eager"
tools/gpu_steps.sh \
 "200 r4p/head512.log env AIMX_HEAD8_MAXF=512 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 100 --timeout-method thread -k 'fused_head or head8'" \
 "200 r4p/c4_base.log $B" \
 "200 r4p/c4_h512.log env AIMX_HEAD8_MAXF=512 $B" \
 "200 r4p/c4_base2.log $B" \
 "200 r4p/c4_h512_r8.log env AIMX_HEAD8_MAXF=512 AIMX_HEAD8_ROWS=8 $B"
