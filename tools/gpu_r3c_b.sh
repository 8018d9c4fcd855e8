#!/bin/bash
# Round 3 (session 3) evidence, part B: c3 / c4 / c5 bench lines (c4 / c5 with their hop roofline),
# the c2 / c4 / c5 step kernel sequences, whole-step MFMA utilisation at c2 / c4 / c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/round; mkdir -p $R
M="--no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
tools/gpu_steps.sh \
  "300 round/bench_c3.log python3 bench.py --config c3 --no-cpu-baseline --no-roofline --no-eager" \
  "400 round/bench_c4.log python3 bench.py --config c4 --no-cpu-baseline" \
  "400 round/bench_c5.log python3 bench.py --config c5 --no-cpu-baseline" || exit $?
for c in c2 c4 c5; do
  tools/gpu_steps.sh "300 round/seq_$c.log rocprofv3 --kernel-trace --output-format csv -d $R/seq_$c -- python3 bench.py --config $c $M" || exit $?
  python3 tools/step_seq.py $R/seq_$c > $R/${c}_seq.txt 2>&1
  rm -rf $R/seq_$c
done
for c in c2 c4 c5; do
  tools/gpu_steps.sh "300 round/${c}_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/${c}_mfma -- python3 bench.py --config $c $M" || exit $?
done
