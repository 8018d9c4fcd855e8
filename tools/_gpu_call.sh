#!/bin/bash
# round-5 working call (overwritten per call): whole GPU suite, smoke, default bench line, c4/c5 lines
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_steps.sh \
 "?900 r5r/tests.log python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread" \
 "300 r5r/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "600 r5r/bench_plain.log python3 bench.py" \
 "300 r5r/bench_c4.log python3 bench.py --config c4 --no-cpu-baseline" \
 "300 r5r/bench_c5.log python3 bench.py --config c5 --no-cpu-baseline"
