#!/bin/bash
# attention-pool rewrite: shape sweep + fixture parity, micro timings, then the whole GPU suite and the bench
set -o pipefail
O=gpurun_out/attn; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention or model_case" -x -q --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1 || { echo "attn tests failed"; tail -40 $O/pytest_attn.log; exit 1; }
tail -2 $O/pytest_attn.log
timeout -k 10 120 python -u tools/attn_micro.py --json $O/attn_micro.json > $O/attn_micro.log 2>&1 || { echo micro failed; tail -20 $O/attn_micro.log; exit 1; }
cat $O/attn_micro.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for c in c2 c4 c5; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline > $O/bench_$c.json 2> $O/bench_$c.err || { echo bench failed; tail -20 $O/bench_$c.err; exit 1; }
tail -1 $O/bench_$c.json | cut -c1-200
done
