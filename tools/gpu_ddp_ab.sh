#!/bin/bash
# 1-GPU A/B of the data-parallel step variants (world-size-1 RCCL group, buckets kept)
set -o pipefail
O=gpurun_out/ddpab; mkdir -p $O
export TMPDIR=/tmp
CFG=${1:-c2}
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config $CFG --steps 30 --warmup 5 --no-cpu-baseline --no-roofline $EXTRA > $O/${CFG}_$n.json 2> $O/${CFG}_$n.err || { echo "$n failed"; tail -5 $O/${CFG}_$n.err; return 1; }
  python -c "import json,sys; d=json.loads(open('$O/${CFG}_$n.json').read().strip().splitlines()[-1]); print('$CFG $n', d['ms_per_step'], d.get('ddp',{}).get('graph_mode'))"
}
EXTRA="" run none AIMX_X=1 && \
EXTRA=--ddp-world1 run capture AIMX_DDP_GRAPH=capture && \
EXTRA=--ddp-world1 run capture_noside AIMX_DDP_GRAPH=capture AIMX_DDP_SIDE=0 && \
EXTRA=--ddp-world1 run split AIMX_DDP_GRAPH=split && \
EXTRA=--ddp-world1 run capture_cl1 AIMX_DDP_GRAPH=capture AIMX_HEAD_CLUSTER=1
