#!/bin/bash
# Round 3: hop roofline / in-step at padded widths (aligned hop.hip path) vs the odd widths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
out=gpurun_out/r3_width.jsonl; : > $out
for h in 512 520 534 1024 1027 1040; do
  c=c4; [ $h -gt 600 ] && c=c5
  timeout -k 10 300 python -u tools/hop_cfg_micro.py --configs $c --hidden $h >> $out || exit 1
done
cat $out
