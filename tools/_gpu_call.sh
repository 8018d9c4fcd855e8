#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4d
tools/gpu_steps.sh \
 "300 r4d/debug_mlps.log python3 -u tools/debug_mlps.py 512 3 512" \
 "?300 r4d/ddp_wrapped.log python3 -u -m pytest tests/test_gpu_ddp.py -v --timeout 200 --timeout-method thread -k 'ddp_wrapped'" \
 "?300 r4d/amp.log python3 -u -m pytest tests/test_gpu_amp.py tests/test_gpu_train.py -v --timeout 200 --timeout-method thread" \
 "?300 r4d/head_gemm_tests.log python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread -k 'head or gemm or c5s or c4s'" \
 "300 r4d/bench_c2.log python3 bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline --no-roofline --no-eager" \
 "300 r4d/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-eager" \
 "300 r4d/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-eager" \
 "300 r4d/c5_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c5_trace -- python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" \
 "120 r4d/seq.log bash -c 'python3 tools/step_seq.py $R/c5_trace > $R/c5_step_seq.txt'"
