#!/bin/bash
# GPU box: -m gpu suite with side-stream weight gradients, then the A/B (AIMX_SIDE_WGRAD=0/1) at c2/c4/c5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/side
tools/gpu_steps.sh "?900 side/tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit $?
tools/gpu_envab.sh c2,c4,c5 default AIMX_SIDE_WGRAD=0
