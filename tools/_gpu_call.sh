#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4o
B="python3 bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline --no-roofline --no-eager"
tools/gpu_steps.sh \
 "400 r4o/tests.log python3 -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_autograph.py -q --timeout 200 --timeout-method thread" \
 "300 r4o/ddp_world1.log python3 bench.py --ddp-world1 --no-cpu-baseline --no-roofline --steps 20" \
 "150 r4o/c2_base.log $B" \
 "150 r4o/c2_wl.log env AIMX_WGRAD_LDS_GEMM=1 $B" \
 "150 r4o/c2_base2.log $B" \
 "150 r4o/c2_wl2.log env AIMX_WGRAD_LDS_GEMM=1 $B" \
 "150 r4o/c2_hop_wc.log env AIMX_HOPR_WC=160 python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-eager" \
 "150 r4o/c4_base.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-eager"
