#!/bin/bash
# round-5 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_steps.sh \
 "?900 r5a/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
 "200 r5a/bench_c2.log python3 bench.py --no-cpu-baseline" \
 "200 r5a/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline" \
 "200 r5a/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline"
