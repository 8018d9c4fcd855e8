#!/bin/bash
# round-2: full GPU suite, attention micro under rocprof, c2/c4/c5 benches
set -o pipefail
O=gpurun_out/r2d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention or adam" -x -q --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1 || { echo "attn tests failed"; tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/attnprof -o run -- python3 tools/attn_micro.py > $O/attnprof.log 2>&1 || { echo prof failed; tail -20 $O/attnprof.log; exit 1; }
for c in c2 c4 c5; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline > $O/bench_$c.json 2> $O/bench_$c.err || { echo bench failed; tail -20 $O/bench_$c.err; exit 1; }
tail -1 $O/bench_$c.json | cut -c1-220
done
