#!/bin/bash
# GEMM 16-byte staging at any alignment: GEMM tests, full suite, c2/c4/c5 benches, c4 profile
set -o pipefail
O=gpurun_out/gemm; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gemm or wgrad" -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1 || { echo "gemm tests failed"; tail -30 $O/pytest_gemm.log; exit 1; }
tail -1 $O/pytest_gemm.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in c2 c4 c5; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline > $O/bench_$c.json 2> $O/bench_$c.err || { echo bench failed; tail -20 $O/bench_$c.err; exit 1; }
tail -1 $O/bench_$c.json | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4prof -o run -- python3 bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/c4prof.log 2>&1 || { echo prof failed; tail -20 $O/c4prof.log; exit 1; }
