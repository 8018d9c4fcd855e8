#!/bin/bash
# GPU box: full -m gpu suite, step-section A/B of the given env settings, then the default bench.
# usage: tools/gpu_ab.sh "ENV=1" ["ENV2=1" ...]
set -o pipefail
envs=""
for e in "$@"; do envs="$envs --env $e"; done
tools/gpu_steps.sh "?600 ab/tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300 ab/sections.log python3 tools/step_sections.py $envs" \
  "300 ab/sections_c4.log python3 tools/step_sections.py --config c4 $envs" \
  "300 ab/bench.log python3 bench.py --no-cpu-baseline --no-roofline"
