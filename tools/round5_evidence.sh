#!/bin/bash
# Round-5 end evidence (GPU box): the hop roofline command under rocprofv3 (kernel stats whose
# k_gather_sum average must agree with the bench line's roofline.ms_per_launch), the c2 FETCH_SIZE /
# WRITE_SIZE passes -> gpurun_out/r5e/hop_traffic.json, the default bench line, c4 / c5 lines, a c2
# step trace, the whole -m gpu suite and smoke. Part a | b | c (one gpurun call each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/r5e; mkdir -p $R
case "$1" in
a) tools/gpu_steps.sh \
    "300 r5e/roof.log python3 bench.py --roofline-only" \
    "300 r5e/roof_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/roof_trace -- python3 bench.py --roofline-only" \
    "200 r5e/fetch.log timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -- python3 bench.py --roofline-only" \
    "200 r5e/write.log timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -- python3 bench.py --roofline-only" \
    "60 r5e/combine.log python3 tools/hop_traffic.py $R/fetch $R/write $R/roof.log $R/hop_traffic.json --kernel k_gather_sum" ;;
b) tools/gpu_steps.sh \
    "500 r5e/bench_c2.log python3 bench.py" \
    "300 r5e/bench_c4.log python3 bench.py --config c4 --no-cpu-baseline" \
    "300 r5e/bench_c5.log python3 bench.py --config c5 --no-cpu-baseline" \
    "300 r5e/c2_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c2_trace -- python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 20 --warmup 5" ;;
c) tools/gpu_steps.sh \
    "?1000 r5e/tests.log python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread" \
    "200 r5e/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" ;;
esac
