#!/bin/bash
# HBM traffic of the odd-width hop (hop_unal.hip) at c4 / c5 roofline size: separate FETCH_SIZE and
# WRITE_SIZE passes of `bench.py --roofline-only --config cN`, combined by tools/hop_traffic.py into
# gpurun_out/traffic/hop_traffic_d{153,307}.json (copied into profiles/ afterwards).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/traffic; mkdir -p $R
for c in c4 c5; do
  d=$([ $c = c4 ] && echo 153 || echo 307)
  tools/gpu_steps.sh \
    "200 traffic/roof_$c.log python3 bench.py --roofline-only --config $c" \
    "200 traffic/fetch_$c.log timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch_$c -- python3 bench.py --roofline-only --config $c" \
    "200 traffic/write_$c.log timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write_$c -- python3 bench.py --roofline-only --config $c" \
    "60 traffic/combine_$c.log python3 tools/hop_traffic.py $R/fetch_$c $R/write_$c gpurun_out/traffic/roof_$c.log $R/hop_traffic_d$d.json --kernel k_gather_unal" || exit $?
done
