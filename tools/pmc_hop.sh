set -o pipefail
R=gpurun_out/hopdiag; mkdir -p $R
tools/gpu_steps.sh \
 "300 hopdiag/micro.log python3 tools/hop_micro.py" \
 "300 hopdiag/gemm.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/gemm -- python3 tools/gemm_micro.py" \
 "600 hopdiag/a.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_READ_sum --output-format csv -d $R/a -- python3 bench.py --roofline-only" \
 "600 hopdiag/b.log rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TD_TC_STALL_sum --output-format csv -d $R/b -- python3 bench.py --roofline-only" \
 "600 hopdiag/c.log rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $R/c -- python3 bench.py --roofline-only" \
 "600 hopdiag/d.log rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum --output-format csv -d $R/d -- python3 bench.py --roofline-only"
