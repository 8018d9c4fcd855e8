#!/bin/bash
# GPU box: the whole -m gpu suite, then the default bench and the step-section timings.
set -o pipefail
tools/gpu_steps.sh "?900 full/tests.log python3 -m pytest tests -m gpu -x -q" \
  "600 full/bench.log python3 bench.py --no-cpu-baseline" \
  "300 full/sections.log python3 tools/step_sections.py"
