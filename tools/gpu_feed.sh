#!/bin/bash
# GPU box: native-feed tests and bench lines (resident vs native C++ collate + H2D per step).
set -o pipefail
tools/gpu_steps.sh "?300 feed/tests.log python3 -u -m pytest tests/test_gpu_feed.py -x -v --timeout 120 --timeout-method thread" \
  "300 feed/bench_native.log python3 bench.py --feed native --no-cpu-baseline --no-roofline" \
  "300 feed/bench_native_eager.log python3 bench.py --feed native --no-graph --no-cpu-baseline --no-roofline" \
  "300 feed/bench_native_c4.log python3 bench.py --config c4 --feed native --no-cpu-baseline --no-roofline" \
  "300 feed/bench_resident.log python3 bench.py --no-cpu-baseline --no-roofline"
