#!/bin/bash
set -o pipefail
O=gpurun_out/attn4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention or model_case" -x -q --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1 || { echo "attn tests failed"; tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/attnprof -o run -- python3 tools/attn_micro.py > $O/attnprof.log 2>&1 || { echo prof failed; tail -20 $O/attnprof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4prof -o run -- python3 bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/c4prof.log 2>&1 || { echo prof failed; tail -20 $O/c4prof.log; exit 1; }
tail -1 $O/c4prof.log | cut -c1-200
