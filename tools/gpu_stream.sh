#!/bin/bash
# HDF5 stream feed benches (c2, c4) + c4 resident step profile + attention parity subset
set -o pipefail
O=gpurun_out/stream; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention" -x -q --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1 || { echo "attn tests failed"; tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
python -m pytest tests/test_h5_stream.py -q -x > $O/pytest_h5.log 2>&1 || { echo "h5 tests failed"; tail -30 $O/pytest_h5.log; exit 1; }
tail -1 $O/pytest_h5.log
for c in c4 c2; do
timeout -k 10 400 python -u bench.py --config $c --feed stream --feed-threads 8 --no-cpu-baseline --no-roofline > $O/bench_${c}_stream.json 2> $O/bench_${c}_stream.err || { echo bench failed; tail -20 $O/bench_${c}_stream.err; exit 1; }
tail -1 $O/bench_${c}_stream.json | cut -c1-200; grep -o '"feed": "[^"]*"' $O/bench_${c}_stream.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4prof -o run -- python3 bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/c4prof.log 2>&1 || { echo prof failed; tail -20 $O/c4prof.log; exit 1; }
