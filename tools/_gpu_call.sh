#!/bin/bash
# round-6 final check at HEAD (overwritten per call): smoke, the whole -m gpu suite, the default
# bench line
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
 "300 r6o/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "?900 r6o/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
 "600 r6o/bench.log python3 bench.py"
