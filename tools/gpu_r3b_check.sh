#!/bin/bash
# Round 3 re-entry: full GPU suite, then c2 / c4 bench lines and the c2 / c4 step kernel sequences.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/r3b; mkdir -p $R
tools/gpu_steps.sh \
  "900 r3b/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "300 r3b/bench_c2.log python bench.py --no-cpu-baseline --no-eager" \
  "400 r3b/bench_c4.log python bench.py --config c4 --no-cpu-baseline --no-eager --no-roofline" || exit $?
for c in c2 c4; do
  tools/gpu_steps.sh "300 r3b/seq_$c.log rocprofv3 --kernel-trace --output-format csv -d $R/$c -- python3 bench.py --config $c --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" || exit $?
  python3 tools/step_seq.py $R/$c > $R/${c}_seq.txt 2>&1
  rm -rf $R/$c
done
