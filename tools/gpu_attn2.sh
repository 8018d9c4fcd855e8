#!/bin/bash
set -o pipefail
O=gpurun_out/attn2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/attn_micro.py --json $O/attn_micro.json > $O/attn_micro.log 2>&1 || { echo micro failed; tail -20 $O/attn_micro.log; exit 1; }
cat $O/attn_micro.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/attn_micro.py > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4prof -o run -- python3 bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $O/c4prof.log 2>&1 || { echo prof failed; tail -20 $O/c4prof.log; exit 1; }
