#!/bin/bash
# Round profile set (run on the GPU box), in parts that each fit one gpurun call:
#   a: the parity tests (a failure stops the set), kernel trace + stats of the default bench command, the hop roofline launches alone, the two
#      PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic, the default bench line;
#   b: the parity tests again, c3/c4/c5 bench lines, step traces of c4/c5, c4's MFMA-busy PMC pass;
#   b2: AMP bench lines (c2/c4/c5), MFMA-busy PMC passes on c2 and c5 (whole-step MFMA against peak);
#   t: smoke and the whole -m gpu suite;
#   s: the c5 1M-molecule 6-hop HDF5 stream line and the feed's own rate at the per-rank thread
#      count of an 8-rank node (16: the box's CPU share per GPU);
#   c: the per-tensor parity report, the DDP lines (world-size-1 RCCL with the DDP-wrapped autograph
#      leg; two gloo ranks sharing the GPU) and smoke;
# Outputs under gpurun_out/round/; tools/collect_profiles.py copies the summaries into profiles/.
# usage: tools/profile_round.sh a|b|b2|c
set -o pipefail
R=gpurun_out/round
mkdir -p $R
A=(
  "300 round/parity.log python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hop_rows.py -q -x --timeout 200 --timeout-method thread"
  "900 round/bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -- python3 bench.py --no-cpu-baseline"
  "600 round/roof.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/roof -- python3 bench.py --roofline-only"
  "60 round/roof_split.log python3 tools/roof_split.py $R/roof $R/roof.log $R/roof_split_c2.json"
  "600 round/roof_c5.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/roof_c5 -- python3 bench.py --config c5 --roofline-only"
  "60 round/roof_split_c5.log python3 tools/roof_split.py $R/roof_c5 $R/roof_c5.log $R/roof_split_c5.json"
  "600 round/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/pmc_fetch -- python3 bench.py --roofline-only"
  "600 round/pmc_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/pmc_write -- python3 bench.py --roofline-only"
  "900 round/bench_plain.log python3 bench.py"
)
B=(
  "300 round/bench_c3.log python3 bench.py --config c3 --no-eager"
  "300 round/bench_c4.log python3 bench.py --config c4 --no-cpu-baseline"
  "300 round/bench_c5.log python3 bench.py --config c5 --no-cpu-baseline"
  "600 round/c4_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c4_trace -- python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
  "600 round/c5_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c5_trace -- python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
  "120 round/seq.log bash -c 'for c in bench c4_trace c5_trace; do python3 tools/step_seq.py $R/\$c > $R/\${c}_step_seq.txt; done'"
  "600 round/c4_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/c4_mfma -- python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
)
B2=(
  "300 round/bench_c2_amp.log python3 bench.py --amp --no-cpu-baseline --no-roofline"
  "300 round/bench_c4_amp.log python3 bench.py --config c4 --amp --no-cpu-baseline --no-roofline"
  "300 round/bench_c5_amp.log python3 bench.py --config c5 --amp --no-cpu-baseline --no-roofline"
  "600 round/c2_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/c2_mfma -- python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
  "600 round/c5_mfma.log rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/c5_mfma -- python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3"
)
S=(
  "900 round/bench_c5_stream.log python3 bench.py --config c5 --feed stream --stream-mols 1000000 --steps 400 --warmup 20 --no-cpu-baseline --no-roofline --no-eager"
  "600 round/feed_rate_c5.log python3 tools/feed_rate.py --config c5 --feed stream --stream-mols 1000000 --batches 400 --threads 16"
)
C=(
  "600 round/c2_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c2_trace -- python3 bench.py --no-cpu-baseline --no-roofline --no-eager --steps 20 --warmup 5"
  "120 round/seq_c2.log bash -c 'python3 tools/step_seq.py $R/c2_trace > $R/c2_trace_step_seq.txt'"
  "600 round/parity_report.log python3 -u tools/parity_report.py --out $R/parity.json"
  "300 round/bench_ddp_world1.log python3 bench.py --ddp-world1 --no-cpu-baseline --no-roofline"
  "300 round/bench_dp2_gloo.log python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-eager"
  "300 round/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'"
)
T=(
  "300 round/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'"
  "?900 round/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread"
)
case "$1" in
  a) tools/gpu_steps.sh "${A[@]}" ;;
  b) tools/gpu_steps.sh "${B[@]}" ;;
  b2) tools/gpu_steps.sh "${B2[@]}" ;;
  c) tools/gpu_steps.sh "${C[@]}" ;;
  s) tools/gpu_steps.sh "${S[@]}" ;;
  t) tools/gpu_steps.sh "${T[@]}" ;;
  *) echo "usage: $0 a|b|c" >&2; exit 2 ;;
esac
