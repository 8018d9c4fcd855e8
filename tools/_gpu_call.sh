#!/bin/bash
# round-5 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -v --timeout 200 --timeout-method thread"
tools/gpu_steps.sh \
 "?400 r5d/ddp.log $T tests/test_gpu_ddp.py tests/test_gpu_autograph.py" \
 "?900 r5d/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
 "300 r5d/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "200 r5d/bench_ddp1.log python3 bench.py --ddp-world1 --no-cpu-baseline --no-roofline" \
 "200 r5d/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline" \
 "200 r5d/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline"
