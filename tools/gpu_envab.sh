#!/bin/bash
# GPU box: bench ms/step for each config under each env setting (A/B), one line per run.
# usage: tools/gpu_envab.sh c2,c4 default X=1 Y=2 ...   (default = no extra env; X=1,Y=2 sets both)
set -o pipefail
cfgs="${1//,/ }"; shift
mkdir -p gpurun_out/envab
out=gpurun_out/envab/summary.txt
for c in $cfgs; do
  for e in "$@"; do
    tag=$(echo "${c}_${e}" | tr -c 'A-Za-z0-9_=\n' '_')
    ev=""; [ "$e" != "default" ] && ev="${e//,/ }"
    timeout -k 10 240 env $ev python3 bench.py --config $c --no-cpu-baseline --no-roofline --no-eager --steps 40 --warmup 10 \
      > gpurun_out/envab/$tag.log 2>&1
    rc=$?
    ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/envab/$tag.log | awk '{print $2}')
    echo "$c $e rc=$rc ms=$ms" | tee -a $out
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/envab/$tag.log; exit $rc; fi
  done
done
