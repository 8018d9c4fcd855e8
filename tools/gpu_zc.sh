#!/bin/bash
# GPU box: parity after the empty-chunk trimming, then the A/B of step sections and bench lines.
set -o pipefail
tools/gpu_steps.sh "?600 zc/tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300 zc/sections.log python3 tools/step_sections.py --env AIMX_NO_ZC=1" \
  "300 zc/bench_c2.log python3 bench.py --no-cpu-baseline --no-roofline" \
  "300 zc/bench_c3.log python3 bench.py --config c3 --no-cpu-baseline --no-roofline" \
  "300 zc/bench_c4.log python3 bench.py --config c4 --no-cpu-baseline --no-roofline" \
  "300 zc/bench_c5.log python3 bench.py --config c5 --no-cpu-baseline --no-roofline"
