#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_steps.sh \
 "60 r4a/mfma4x4.log tools/micro/mfma4x4" \
 "?300 r4a/head_mlps_tests.log python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'fused_head or streamed_mlp_matches_per_gemm'" \
 "?400 r4a/mlps_model.log python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'full_size or c4s or c5s or streamed_mlp_forced or test_model_case'" \
 "300 r4a/bench_c2.log python3 bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline --no-roofline --no-eager" \
 "300 r4a/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-eager" \
 "300 r4a/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-eager" \
 "?900 r4a/tests.log python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
 "400 r4a/dp2_gloo.log python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline --no-roofline"
