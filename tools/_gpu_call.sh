#!/bin/bash
# round-6 working call (overwritten per call): the whole -m gpu suite on the pruned product library,
# hop rooflines after the row-range cap fix, c2 / c4 / c5 bench lines
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
 "?900 r6g/tests.log python3 -u -m pytest -q --maxfail 10 --timeout 200 --timeout-method thread tests -m gpu" \
 "200 r6g/roof_c5.log python3 bench.py --config c5 --roofline-only" \
 "200 r6g/roof_c4.log python3 bench.py --config c4 --roofline-only" \
 "200 r6g/roof_c2.log python3 bench.py --roofline-only" \
 "300 r6g/c5.log python3 bench.py --config c5 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6g/c4.log python3 bench.py --config c4 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6g/c2.log python3 bench.py --no-cpu-baseline --no-eager --no-roofline"
