#!/bin/bash
# Round 3: c2 native-feed trace (kernels + copies) for step gaps; head cluster A/B at world 1 with
# the RCCL group (the multi-rank setting forces cluster 1); hop roofline traces at c4 / c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r3_misc; mkdir -p $R
S=("300 r3_misc/c2n_trace.log rocprofv3 --kernel-trace --memory-copy-trace -d $R/c2n -o c2n -- python3 bench.py --feed native --steps 60 --warmup 10 --no-cpu-baseline --no-roofline --no-eager")
S+=("300 r3_misc/c2r_trace.log rocprofv3 --kernel-trace -d $R/c2r -o c2r -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-roofline --no-eager")
for cl in 1 2; do
  S+=("300 r3_misc/ddp1_cluster$cl.log env AIMX_HEAD_CLUSTER=$cl python3 bench.py --ddp-world1 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --no-eager")
done
for c in c4 c5; do
  S+=("300 r3_misc/roof_$c.log rocprofv3 --kernel-trace --output-format csv -d $R/roof_$c -- python3 bench.py --config $c --roofline-only")
done
tools/gpu_steps.sh "${S[@]}"
