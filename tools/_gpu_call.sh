#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4i
tools/gpu_steps.sh \
 "120 r4i/mlps_trace_c4.log python3 -u tools/mlps_trace.py c4" \
 "120 r4i/mlps_trace_c5.log python3 -u tools/mlps_trace.py c5" \
 "?900 r4i/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread"
