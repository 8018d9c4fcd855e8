#!/bin/bash
# round-5 working call (overwritten per call): padded F / UG row strides (16-byte rows) — parity, then A/B
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -v --timeout 200 --timeout-method thread"
B="python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 30 --warmup 8"
tools/gpu_steps.sh \
 "400 r5l/parity.log $T tests/test_gpu_parity.py -k 'full_size or c4s or c5s or shell_layer or mlp or stack or case'" \
 "300 r5l/c5_pad.log $B --config c5" \
 "300 r5l/c5_dense.log env AIMX_STACK_PAD=0 $B --config c5" \
 "300 r5l/c4_pad.log $B --config c4" \
 "300 r5l/c4_dense.log env AIMX_STACK_PAD=0 $B --config c4" \
 "300 r5l/c2_pad.log $B"
