#!/bin/bash
# GPU box: per-step kernel sequence of one bench configuration. usage: tools/gpu_seqx.sh TAG [bench args...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
R=gpurun_out/seqx
mkdir -p $R
tools/gpu_steps.sh "300 seqx/$tag.log rocprofv3 --kernel-trace --output-format csv -d $R/$tag -- python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3 $*" || exit $?
python3 tools/step_seq.py $R/$tag > $R/${tag}_seq.txt 2>&1
rm -rf $R/$tag
tail -1 $R/${tag}_seq.txt
