#!/bin/bash
# round-6 working call (overwritten per call): the deep-K head GEMM at 16 / 8 waves vs the tiles,
# the r6c failures, c5 / c4 / c2 bench lines with the large-tile GEMM off by default, c5 trace
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python3 -u -m pytest -q --timeout 200 --timeout-method thread"
TL=aimnet-x2d_amd/lib/libaimx_tune.so
B="bench.py --config c5 --steps 10 --warmup 5 --no-cpu-baseline --no-eager --no-roofline"
tools/gpu_steps.sh \
 "?600 r6e/tests.log $T --maxfail 8 tests/test_gpu_parity.py::test_gemm_deep_kernel tests/test_gpu_parity.py::test_gemm_few_rows_deep_k tests/test_gpu_hop_rows.py tests/test_gpu_autograph.py tests/test_gpu_train.py::test_large_batch_past_2gib_equals_two_batches" \
 "200 r6e/deep16.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP=16 python3 tools/gemm_micro.py deep" \
 "200 r6e/deep8.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP=8 python3 tools/gemm_micro.py deep" \
 "200 r6e/deep0.log AIMX_LIB_PATH=$TL AIMX_GEMM_DEEP=0 python3 tools/gemm_micro.py deep" \
 "300 r6e/c5.log python3 bench.py --config c5 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6e/c4.log python3 bench.py --config c4 --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6e/c2.log python3 bench.py --no-cpu-baseline --no-eager --no-roofline" \
 "300 r6e/prof_c5.log rocprofv3 --kernel-trace --stats -d gpurun_out/r6e/prof_c5 -o run -- python3 $B"
