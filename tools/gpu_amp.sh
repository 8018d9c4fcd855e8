#!/bin/bash
# GPU box: AMP tests + fp32 parity suite, then fp32 vs AMP bench lines for c2/c4/c5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/amp
tools/gpu_steps.sh "?900 amp/tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300 amp/c2.log python3 bench.py --amp --no-cpu-baseline --no-roofline" \
  "300 amp/c4.log python3 bench.py --amp --config c4 --no-cpu-baseline --no-roofline" \
  "300 amp/c5.log python3 bench.py --amp --config c5 --no-cpu-baseline --no-roofline" \
  "300 amp/c4_32.log python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager" \
  "300 amp/c5_32.log python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager"
