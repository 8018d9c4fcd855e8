#!/bin/bash
# Round 3 (session 3) evidence, part A: full GPU suite, smoke, default bench under rocprofv3,
# hop roofline kernel stats and the two HBM PMC passes, the plain default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
rm -rf gpurun_out/round; mkdir -p gpurun_out/round
tools/gpu_steps.sh \
  "900 round/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "300 round/smoke.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" || exit $?
R=gpurun_out/round
tools/gpu_steps.sh \
  "900 round/bench.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/bench -- python3 bench.py --no-cpu-baseline" \
  "600 round/roof.log rocprofv3 --kernel-trace --stats --output-format csv -d $R/roof -- python3 bench.py --roofline-only" \
  "600 round/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/pmc_fetch -- python3 bench.py --roofline-only" \
  "600 round/pmc_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/pmc_write -- python3 bench.py --roofline-only" \
  "900 round/bench_plain.log python3 bench.py"
