#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4g
tools/gpu_steps.sh \
 "?400 r4g/tests.log python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograph.py -v --timeout 200 --timeout-method thread" \
 "?200 r4g/head.log python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 100 --timeout-method thread -k head" \
 "150 r4g/bench_c2.log python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline" \
 "250 r4g/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline" \
 "250 r4g/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline"
