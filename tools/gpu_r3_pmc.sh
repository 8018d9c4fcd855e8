#!/bin/bash
# Round 3 PMC set: hop roofline HBM traffic at D = 153 / 307 (c4 / c5: FETCH_SIZE and WRITE_SIZE,
# one counter per pass) and whole-step MFMA busy at c2 / c4 / c5. Summaries under gpurun_out/r3_pmc.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=gpurun_out/r3_pmc
mkdir -p $R
S=()
for c in c4 c5; do
  S+=("300 r3_pmc/roof_$c.log python3 bench.py --config $c --roofline-only")
  S+=("300 r3_pmc/fetch_$c.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch_$c -- python3 bench.py --config $c --roofline-only")
  S+=("300 r3_pmc/write_$c.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write_$c -- python3 bench.py --config $c --roofline-only")
done
for c in c2 c4 c5; do
  S+=("300 r3_pmc/mfma_$c.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/mfma_$c -- python3 bench.py --config $c --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3")
done
tools/gpu_steps.sh "${S[@]}" || exit $?
python3 tools/hop_traffic.py $R/fetch_c4 $R/write_c4 gpurun_out/r3_pmc/roof_c4.log $R/hop_traffic_d153.json --kernel k_gather_rows
python3 tools/hop_traffic.py $R/fetch_c5 $R/write_c5 gpurun_out/r3_pmc/roof_c5.log $R/hop_traffic_d307.json --kernel k_gather_rows
for c in c2 c4 c5; do python3 tools/mfma_summary.py $R/mfma_$c 12 > $R/mfma_$c.txt; head -3 $R/mfma_$c.txt; done
