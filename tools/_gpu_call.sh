#!/bin/bash
# round-5 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -v --timeout 200 --timeout-method thread"
tools/gpu_steps.sh \
 "?600 r5e/ddp.log $T tests/test_gpu_ddp.py tests/test_gpu_autograph.py tests/test_gpu_stream.py tests/test_gpu_parity.py -k 'ddp or autograph or stream or full_size'" \
 "200 r5e/bench_ddp1.log python3 bench.py --ddp-world1 --no-cpu-baseline --no-roofline"
