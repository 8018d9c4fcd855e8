#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4m
tools/gpu_steps.sh \
 "300 r4m/parity.log python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hop_rows.py -q -x --timeout 200 --timeout-method thread" \
 "120 r4m/trace_c4.log python3 -u tools/mlps_trace.py c4" \
 "120 r4m/trace_c5.log python3 -u tools/mlps_trace.py c5" \
 "150 r4m/bench_c2.log python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --no-eager" \
 "200 r4m/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline" \
 "200 r4m/bench_c4_wl.log env AIMX_WGRAD_LDS_GEMM=1 python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline --no-eager" \
 "200 r4m/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline" \
 "200 r4m/bench_c5_wl.log env AIMX_WGRAD_LDS_GEMM=1 python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline --no-eager"
