#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4f
tools/gpu_steps.sh \
 "200 r4f/debug_ddp.log python3 -u tools/debug_ddp_wrapped.py" \
 "?500 r4f/tests.log python3 -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograph.py tests/test_gpu_ddp.py -v --timeout 200 --timeout-method thread" \
 "?200 r4f/head.log python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 100 --timeout-method thread -k head" \
 "120 r4f/bench_c2.log python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --no-eager" \
 "300 r4f/c4e_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c4e_trace -- python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager --no-graph --steps 10 --warmup 3"
