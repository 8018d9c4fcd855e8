#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4h
B="python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-eager"
tools/gpu_steps.sh \
 "?400 r4h/tests.log python3 -u -m pytest tests/test_gpu_train.py -v --timeout 200 --timeout-method thread" \
 "?200 r4h/head.log python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 100 --timeout-method thread -k head" \
 "150 r4h/bench_c2.log python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline" \
 "250 r4h/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline" \
 "250 r4h/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline" \
 "120 r4h/pmc_a.log timeout -s KILL 110 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/pmc_a -- $B" \
 "120 r4h/pmc_b.log timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/pmc_b -- $B" \
 "60 r4h/pmc_sum.log bash -c 'for k in k_mlps_fwd k_mlps_bwd k_wgrad_lds k_gemm; do echo == \$k; python3 tools/pmc_summary.py $R/pmc_a \$k; python3 tools/pmc_summary.py $R/pmc_b \$k; done'"
