#!/bin/bash
# round-4 working call (overwritten per call)
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r4l
tools/gpu_steps.sh \
 "300 r4l/parity.log python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hop_rows.py -q -x --timeout 200 --timeout-method thread" \
 "120 r4l/trace_c4.log python3 -u tools/mlps_trace.py c4" \
 "120 r4l/trace_c5.log python3 -u tools/mlps_trace.py c5" \
 "120 r4l/wtrace_c4.log python3 -u tools/wgrad_trace.py c4" \
 "120 r4l/wtrace_c5.log python3 -u tools/wgrad_trace.py c5" \
 "200 r4l/bench_c4.log python3 bench.py --config c4 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline" \
 "200 r4l/bench_c5.log python3 bench.py --config c5 --steps 30 --warmup 8 --no-cpu-baseline --no-roofline" \
 "300 r4l/c5_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c5_trace -- python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" \
 "120 r4l/seq.log bash -c 'python3 tools/step_seq.py $R/c5_trace > $R/c5_step_seq.txt'"
