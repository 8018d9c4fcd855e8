#!/bin/bash
set -o pipefail
O=gpurun_out/abl; mkdir -p $O
export TMPDIR=/tmp
for a in 0 1 2 3 4; do
  AIMX_LIB_PATH=$PWD/aimnet-x2d_amd/lib/libaimx_abl.so AIMX_ATTN_ABL=$a timeout -k 10 120 python -u tools/attn_micro.py > $O/abl$a.log 2>&1 || { echo "abl $a failed"; tail -20 $O/abl$a.log; exit 1; }
  echo "== abl $a"; grep config $O/abl$a.log | cut -c1-110
done
