#!/bin/bash
# round-6 final refresh (overwritten per call): smoke + the whole -m gpu suite, c4 / c5 lines, step
# traces and MFMA passes after the head-path and weight-gradient split changes; the parity report's
# c4 cases (their head now runs the module path)
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=gpurun_out/round
mkdir -p $R
tools/gpu_steps.sh \
 "300 round/smoke.log python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "?900 round/tests.log python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread" \
 "300 round/bench_c4.log python3 bench.py --config c4 --no-cpu-baseline" \
 "300 round/bench_c5.log python3 bench.py --config c5 --no-cpu-baseline" \
 "300 round/c4_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c4_trace -- python3 bench.py --config c4 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" \
 "300 round/c5_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/c5_trace -- python3 bench.py --config c5 --no-cpu-baseline --no-roofline --no-eager --steps 10 --warmup 3" \
 "120 round/seq.log bash -c 'for c in c4_trace c5_trace; do python3 tools/step_seq.py $R/\$c > $R/\${c}_step_seq.txt; done'" \
 "300 round/parity_report_c4.log python3 -u tools/parity_report.py --out $R/parity_c4.json c4s c4"
