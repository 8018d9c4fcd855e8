#!/bin/bash
# round-5 working call (overwritten per call): register-file hop kernel, parity then speed
export PYTHONDONTWRITEBYTECODE=1
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
M="python3 tools/hop_cfg_micro.py --configs c4,c5"
tools/gpu_steps.sh \
 "?200 r5h/skinny_tests.log $T tests/test_gpu_parity.py -k 'skinny or gemm or wgrad or activation_epilogue or linear'" \
 "?300 r5h/hop_tests.log $T tests/test_gpu_hop_rows.py" \
 "200 r5h/regs.log $M" \
 "200 r5h/rows.log env AIMX_HOP_REGS=0 $M" \
 "200 r5h/wlib_c5.log python3 tools/wgrad_lib_ab.py c5" \
 "200 r5h/wlib_c4.log python3 tools/wgrad_lib_ab.py c4" \
 "200 r5h/gemm_head.log python3 tools/gemm_micro.py head" \
 "200 r5h/gemm_head0.log env AIMX_SKINNY=0 python3 tools/gemm_micro.py head" \
 "400 r5h/model.log $T tests/test_gpu_parity.py -k 'full_size or c4s or c5s or stereo'"
