#!/bin/bash
# Hop kernel tuning sweep (GPU box): parity of the hop tests, then ONE tools/hop_micro.py process
# comparing the given AIMX_HOP_* settings interleaved (2 rounds). Logs under gpurun_out/hs/.
set -o pipefail
mkdir -p gpurun_out/hs
args=()
for cfg in "$@"; do args+=(--env "$cfg"); done
tools/gpu_steps.sh "?400 hs/tests.log python3 -m pytest tests/test_gpu_parity.py -m gpu -x -q -k hop" && \
timeout -k 10 600 python3 tools/hop_micro.py --rounds 2 "${args[@]}" > gpurun_out/hs/micro.log 2>&1
