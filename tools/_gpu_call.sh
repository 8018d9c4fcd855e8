#!/bin/bash
# round-5 working call (overwritten per call): padded F / UG / R, A row strides — parity, then A/B
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -v --timeout 200 --timeout-method thread"
B="python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 30 --warmup 8"
tools/gpu_steps.sh \
 "400 r5m/parity.log $T tests/test_gpu_parity.py -k 'full_size or c4s or c5s or shell_layer or mlp or stack or case or c1 or trajectory'" \
 "300 r5m/c5_pad.log $B --config c5" \
 "300 r5m/c4_pad.log $B --config c4" \
 "300 r5m/c2_pad.log $B" \
 "300 r5m/c3_pad.log $B --config c3"
