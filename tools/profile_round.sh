#!/bin/bash
# Round profile set (run on the GPU box): kernel trace + stats of the default bench command, the
# hop roofline launches alone, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.
# Outputs under gpurun_out/round/; tools/collect_profiles.py copies the summaries into profiles/.
# Extra (after the core set): the c3/c4/c5 bench lines (fp32 and AMP) and MFMA-busy PMC passes on
# c2, c4 and c5 (whole-step MFMA utilisation against chip peak).
set -o pipefail
# usage: tools/profile_round.sh [FIRST]  (FIRST: 0-based index of the first step to run, to resume)
R=gpurun_out/round
mkdir -p $R
STEPS=(
  "900 round/bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -- python3 bench.py --no-cpu-baseline"
  "600 round/roof.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/roof -- python3 bench.py --roofline-only"
  "600 round/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/pmc_fetch -- python3 bench.py --roofline-only"
  "600 round/pmc_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/pmc_write -- python3 bench.py --roofline-only"
  "900 round/bench_plain.log python3 bench.py"
  "300 round/bench_c3.log python3 bench.py --config c3 --no-cpu-baseline --no-roofline --no-eager"
  "300 round/bench_c4.log python3 bench.py --config c4 --no-cpu-baseline"
  "300 round/bench_c5.log python3 bench.py --config c5 --no-cpu-baseline"
  "300 round/bench_c2_amp.log python3 bench.py --amp --no-cpu-baseline --no-roofline"
  "300 round/bench_c4_amp.log python3 bench.py --config c4 --amp --no-cpu-baseline --no-roofline"
  "300 round/bench_c5_amp.log python3 bench.py --config c5 --amp --no-cpu-baseline --no-roofline"
  "120 round/counters.log rocprofv3 -L"
  "600 round/c4_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c4_trace -- python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
  "600 round/c2_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/c2_mfma -- python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
  "600 round/c4_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/c4_mfma -- python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
  "600 round/c5_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/c5_mfma -- python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
)
tools/gpu_steps.sh "${STEPS[@]:${1:-0}}"
