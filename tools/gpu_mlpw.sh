#!/bin/bash
# GPU box: -m gpu suite, the weight-resident MLP trace, the MLP-path A/B at c1/c2/c3 and the c2 sequence.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
tools/gpu_steps.sh "?900 diag/tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 diag/mlpw_trace.log env AIMX_LIB_PATH=aimnet-x2d_amd/lib_trace/libaimx.so python3 tools/mlpw_trace.py" || exit $?
tools/gpu_envab.sh c1,c2,c3 default AIMX_MLPW=0 && tools/gpu_seqx.sh c2w
