#!/bin/bash
# Full GPU test suite (one process), log under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_full.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r3_gpu_full.log | tail -5
tail -3 gpurun_out/r3_gpu_full.log
exit $rc
