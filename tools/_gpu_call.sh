#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4n
tools/gpu_steps.sh \
 "300 r4n/parity.log python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k 'wgrad or model_case or full_size or gemm'" \
 "120 r4n/wtrace_c4.log python3 -u tools/wgrad_trace.py c4" \
 "150 r4n/bench_c2.log python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --no-eager" \
 "200 r4n/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline --no-eager" \
 "200 r4n/bench_c4_bb64.log env AIMX_WGRAD_BB=64 python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline --no-eager" \
 "200 r4n/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline --no-eager" \
 "200 r4n/bench_c5_bb64.log env AIMX_WGRAD_BB=64 python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline --no-eager" \
 "150 r4n/bench_c2_bb64.log env AIMX_WGRAD_BB=64 python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --no-eager"
