#!/bin/bash
# GPU box: the whole -m gpu suite, the default bench line, and the c2 per-step kernel sequence.
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/check
mkdir -p $R
tools/gpu_steps.sh "?900 check/tests.log python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "400 check/bench.log python3 bench.py --no-cpu-baseline" \
  "300 check/c2trace.log rocprofv3 --kernel-trace --output-format csv -d $R/c2 -- python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" || exit $?
python3 tools/step_seq.py $R/c2 > $R/c2_seq.txt 2>&1
rm -rf $R/c2
tail -1 $R/c2_seq.txt
