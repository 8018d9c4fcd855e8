#!/bin/bash
# round-6 working call (overwritten per call): the fused post-pool head against the module path
# (deep-K GEMMs) at c4 and c2; c5 / c4 / c2 lines at the new weight-gradient split default
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TL=aimnet-x2d_amd/lib/libaimx_tune.so
A="--no-cpu-baseline --no-eager --no-roofline"
tools/gpu_steps.sh \
 "300 r6l/c4_fused.log python3 bench.py --config c4 $A" \
 "300 r6l/c4_module.log python3 tools/ab_module_head.py --config c4 $A" \
 "300 r6l/c2_fused.log python3 bench.py $A" \
 "300 r6l/c2_module.log python3 tools/ab_module_head.py $A" \
 "300 r6l/c2_module_k256.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP_KMIN=256 python3 tools/ab_module_head.py $A" \
 "300 r6l/c5.log python3 bench.py --config c5 $A"
