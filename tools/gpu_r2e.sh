#!/bin/bash
# GPU box (round 2 re-entry): whole -m gpu suite, default bench, eager c2 bench.
set -o pipefail
tools/gpu_steps.sh "?900 r2e/tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300 r2e/bench.log python3 bench.py --no-cpu-baseline" \
  "300 r2e/eager.log python3 bench.py --no-graph --no-cpu-baseline --no-roofline --steps 30"
