#!/bin/bash
# Round profile set (run on the GPU box): kernel trace + stats of the default bench command, the
# hop roofline launches alone, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.
# Outputs under gpurun_out/round/; tools/collect_profiles.py copies the summaries into profiles/.
set -o pipefail
R=gpurun_out/round
mkdir -p $R
tools/gpu_steps.sh \
  "900 round/bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -- python3 bench.py --no-cpu-baseline" \
  "600 round/roof.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/roof -- python3 bench.py --roofline-only" \
  "600 round/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/pmc_fetch -- python3 bench.py --roofline-only" \
  "600 round/pmc_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/pmc_write -- python3 bench.py --roofline-only" \
  "900 round/bench_plain.log python bench.py"
