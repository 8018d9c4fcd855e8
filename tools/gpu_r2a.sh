#!/bin/bash
# round-2 GPU pass: tests, parity report, DDP capture/split A/B at world 1, rocprof of the bench
set -o pipefail
O=gpurun_out/r2b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/parity_report.py --out $O/parity.json > $O/parity.log 2>&1 || { echo parity failed; tail -20 $O/parity.log; exit 1; }
cat $O/parity.log
for m in capture split; do
  AIMX_DDP_GRAPH=$m timeout -k 10 200 python bench.py --steps 30 --warmup 5 --ddp-world1 --no-cpu-baseline --no-roofline > $O/ddp_$m.json 2> $O/ddp_$m.err || { echo "ddp $m failed"; tail -20 $O/ddp_$m.err; exit 1; }
  tail -1 $O/ddp_$m.json
done
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline > $O/plain.json 2>&1 && tail -1 $O/plain.json
