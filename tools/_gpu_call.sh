#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4e
tools/gpu_steps.sh \
 "?400 r4e/parity.log python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hop_rows.py -q --timeout 200 --timeout-method thread" \
 "200 r4e/debug_ddp.log python3 -u tools/debug_ddp_wrapped.py" \
 "120 r4e/bench_c2_r8.log python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --no-eager" \
 "120 r4e/bench_c2_r4.log env AIMX_HEAD8_ROWS=4 python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline --no-eager" \
 "200 r4e/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline" \
 "200 r4e/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline" \
 "300 r4e/c4_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c4_trace -- python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" \
 "300 r4e/c5_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c5_trace -- python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" \
 "120 r4e/seq.log bash -c 'for c in c4 c5; do python3 tools/step_seq.py $R/\${c}_trace > $R/\${c}_step_seq.txt; done'" \
 "?300 r4e/head4_tests.log env AIMX_HEAD8_ROWS=4 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k 'fused_head or model_case'" \
 "?900 r4e/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread"
