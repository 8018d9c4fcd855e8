#!/bin/bash
# GPU box: head phase trace (variant build), eager host profile, weight-gradient KPER sweeps at c4/c5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
tools/gpu_steps.sh "200 diag/head_trace.log env AIMX_LIB_PATH=aimnet-x2d_amd/lib_trace/libaimx.so HEAD_CLUSTERS=1,2,4 python3 tools/head_trace.py" \
  "300 diag/eager_prof.log python3 tools/eager_profile.py" \
  "300 diag/wgrad_c4.log python3 tools/wgrad_micro.py c4 0,256,1024,2048" \
  "300 diag/wgrad_c5.log python3 tools/wgrad_micro.py c5 0,256,1024,2048" \
  "300 diag/wgrad_c2.log python3 tools/wgrad_micro.py c2 0,256,1024"
