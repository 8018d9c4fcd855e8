#!/bin/bash
# round-5 working call (overwritten per call): head tiles 32x32, one MLP pack launch per direction, row copy
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -v --timeout 200 --timeout-method thread"
B="python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 30 --warmup 8"
tools/gpu_steps.sh \
 "400 r5q/parity.log $T tests/test_gpu_parity.py -k 'full_size or c4s or c5s or shell_layer or stack or case or gemm or head'" \
 "300 r5q/c5.log $B --config c5" \
 "300 r5q/c4.log $B --config c4" \
 "300 r5q/c2.log $B"
