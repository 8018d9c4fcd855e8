#!/bin/bash
# round-5 working call (overwritten per call): lone weight-gradient split target A/B on the c2 step
export PYTHONDONTWRITEBYTECODE=1
B="python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 200 --warmup 20"
tools/gpu_steps.sh \
 "300 r5v/c2_1152.log $B" \
 "300 r5v/c2_384.log env AIMX_WGRAD_WGS=384 $B" \
 "300 r5v/c2_768.log env AIMX_WGRAD_WGS=768 $B" \
 "300 r5v/c2_2048.log env AIMX_WGRAD_WGS=2048 $B" \
 "300 r5v/c4_1152.log $B --config c4" \
 "300 r5v/c4_384.log env AIMX_WGRAD_WGS=384 $B --config c4"
