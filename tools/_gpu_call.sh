#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4q
tools/gpu_steps.sh \
 "?900 r4q/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
 "200 r4q/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline" \
 "300 r4q/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "200 r4q/bench_c2.log python3 bench.py --no-cpu-baseline"
