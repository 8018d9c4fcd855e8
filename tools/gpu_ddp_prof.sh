#!/bin/bash
set -o pipefail
O=gpurun_out/ddpprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for side in 1 0; do
  AIMX_DDP_GRAPH=capture AIMX_DDP_SIDE=$side timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/side$side -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --ddp-world1 > $O/side$side.log 2>&1 || { echo fail $side; tail -20 $O/side$side.log; exit 1; }
done
find $O -name "*stats*" | head
