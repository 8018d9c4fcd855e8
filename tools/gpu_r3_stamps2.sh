#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
: > gpurun_out/r3_stamps2.jsonl
for d in 0 1 4 5 2 3; do
  echo "dbg=$d" >> gpurun_out/r3_stamps2.jsonl
  AIMX_HOPR_DBG=$d AIMX_LIB_PATH=aimnet-x2d_amd/lib_stamps/libaimx.so timeout -k 10 300 python -u tools/hop_stamps.py --config c4 --atoms 0 >> gpurun_out/r3_stamps2.jsonl 2>&1 || { cat gpurun_out/r3_stamps2.jsonl; exit 1; }
done
grep -E "dbg|in_step" gpurun_out/r3_stamps2.jsonl
