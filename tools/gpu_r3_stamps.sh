#!/bin/bash
# Round 3: phase stamps of hop_rows.hip (diagnostic library built here, -DAIMX_HOPR_STAMPS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
: > gpurun_out/r3_stamps.jsonl
for c in ${CFGS:-c4 c5}; do
  AIMX_LIB_PATH=aimnet-x2d_amd/lib_stamps/libaimx.so timeout -k 10 300 python -u tools/hop_stamps.py --config $c >> gpurun_out/r3_stamps.jsonl 2>&1 || { cat gpurun_out/r3_stamps.jsonl; exit 1; }
done
grep case gpurun_out/r3_stamps.jsonl
