#!/bin/bash
set -o pipefail
O=gpurun_out/attn3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention or model_case" -x -q --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1 || { echo "attn tests failed"; tail -40 $O/pytest_attn.log; exit 1; }
tail -2 $O/pytest_attn.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/attn_micro.py > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
grep config $O/prof.log | cut -c1-120
