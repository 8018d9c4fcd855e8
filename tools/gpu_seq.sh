#!/bin/bash
# GPU box: kernel traces of short c2/c4/c5 bench runs (per-step kernel sequence via tools/step_seq.py).
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/seq
mkdir -p $R
for c in c2 c4 c5; do
  tools/gpu_steps.sh "300 seq/$c.log rocprofv3 --kernel-trace --output-format csv -d $R/$c -- python3 bench.py --config $c --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" || exit $?
  python3 tools/step_seq.py $R/$c > $R/${c}_seq.txt 2>&1
  rm -rf $R/$c
done
