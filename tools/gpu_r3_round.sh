#!/bin/bash
# Round 3 evidence set: full GPU suite, smoke(), the default bench line, its rocprof kernel trace,
# the c3/c4/c5 lines, and the hop roofline kernel trace. Outputs under gpurun_out/r3_round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r3_round; mkdir -p $R
tools/gpu_steps.sh \
  "900 r3_round/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "300 r3_round/smoke.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "600 r3_round/bench_default.log python bench.py" \
  "600 r3_round/bench_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench_trace -- python3 bench.py --no-cpu-baseline --no-eager" \
  "300 r3_round/bench_c3.log python bench.py --config c3 --no-cpu-baseline --no-roofline --no-eager" \
  "400 r3_round/bench_c4.log python bench.py --config c4 --no-cpu-baseline --no-eager" \
  "400 r3_round/bench_c5.log python bench.py --config c5 --no-cpu-baseline --no-eager" \
  "400 r3_round/bench_c2_stream.log python bench.py --config c2 --feed stream --steps 300 --warmup 20 --no-cpu-baseline --no-roofline --no-eager" \
  "600 r3_round/bench_c4_stream1m.log python bench.py --config c4 --feed stream --stream-mols 1000000 --steps 400 --warmup 20 --no-cpu-baseline --no-roofline --no-eager" \
  "400 r3_round/roof_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/roof_trace -- python3 bench.py --roofline-only"
rc=$?
rm -f /tmp/aimx_stream_*.h5
exit $rc
