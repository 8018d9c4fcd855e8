#!/bin/bash
# round-6 working call (overwritten per call): [Wi; Wg] GEMMs at the reference's odd weight row stride
# vs a 4-float-rounded stride (16-byte staging), c4 / c5 shapes
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
 "200 r6h/ugpad.log python3 tools/gemm_micro.py ugpad"
