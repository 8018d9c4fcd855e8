#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_steps.sh \
 "300 r4b/debug_mlps.log python3 -u tools/debug_mlps.py 512 3 512" \
 "?600 r4b/tests_fix.log python3 -u -m pytest tests/test_gpu_autograph.py tests/test_gpu_ddp.py tests/test_gpu_train.py tests/test_gpu_amp.py -v --timeout 200 --timeout-method thread"
