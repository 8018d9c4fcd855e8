#!/bin/bash
# round-5 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
B="python3 bench.py --no-cpu-baseline --no-roofline --steps 40 --warmup 8"
tools/gpu_steps.sh \
 "200 r5f/ddp1.log python3 bench.py --ddp-world1 --no-cpu-baseline --no-roofline" \
 "200 r5f/c2_q128.log env AIMX_BENCH_QUANTUM=128 $B" \
 "200 r5f/c2_q64.log env AIMX_BENCH_QUANTUM=64 $B" \
 "200 r5f/c2_q32.log env AIMX_BENCH_QUANTUM=32 $B" \
 "200 r5f/c5_q128.log env AIMX_BENCH_QUANTUM=128 $B --config c5" \
 "200 r5f/c5_q64.log env AIMX_BENCH_QUANTUM=64 $B --config c5" \
 "200 r5f/c5_q32.log env AIMX_BENCH_QUANTUM=32 $B --config c5" \
 "200 r5f/c4_q128.log env AIMX_BENCH_QUANTUM=128 $B --config c4" \
 "200 r5f/c4_q64.log env AIMX_BENCH_QUANTUM=64 $B --config c4" \
 "200 r5f/c4_q32.log env AIMX_BENCH_QUANTUM=32 $B --config c4"
