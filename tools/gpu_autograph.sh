#!/bin/bash
# GPU box: autograph tests, the eager probe with and without autograph, and the c2 bench line
# (eager and eager+autograph rates).
set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh "300 ag/tests.log python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_autograph.py" \
  "200 ag/probe_ag.log env AIMX_AUTOGRAPH=1 python3 tools/eager_sync_probe.py" \
  "300 ag/bench.log python3 bench.py --no-cpu-baseline --no-roofline"
