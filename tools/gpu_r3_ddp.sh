#!/bin/bash
# Round 3: data-parallel self-checks (fallback, DDP-wrapped drop-in, checksums), autograph/Adam
# additions, and a --ddp-world1 bench line carrying the new ddp fields.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py \
  tests/test_gpu_autograph.py tests/test_gpu_parity.py -k "ddp or rccl or autograph or adam or pad_batch" \
  > gpurun_out/r3_ddp_tests.log 2>&1 || { tail -60 gpurun_out/r3_ddp_tests.log; exit 1; }
tail -3 gpurun_out/r3_ddp_tests.log
timeout -k 10 300 python -u bench.py --ddp-world1 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-eager \
  > gpurun_out/r3_bench_ddp_world1.json 2> gpurun_out/r3_bench_ddp_world1.err; echo "ddp-world1 rc=$?"
tail -c 1200 gpurun_out/r3_bench_ddp_world1.json
