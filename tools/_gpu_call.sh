#!/bin/bash
# round-5 working call (overwritten per call): skinny GEMM stages A/B
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
tools/gpu_steps.sh \
 "?200 r5i/skinny_tests.log $T tests/test_gpu_parity.py -k 'skinny or gemm or wgrad or linear'" \
 "200 r5i/head_ns4.log python3 tools/gemm_micro.py head" \
 "200 r5i/head_ns2.log env AIMX_SKINNY_NS=2 python3 tools/gemm_micro.py head" \
 "200 r5i/head_off.log env AIMX_SKINNY=0 python3 tools/gemm_micro.py head" \
 "300 r5i/c5_ns4.log python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 30 --warmup 8" \
 "300 r5i/c5_off.log env AIMX_SKINNY=0 python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 30 --warmup 8"
