#!/bin/bash
# Round 3: Adam fold / autograph gate tests, then resident vs native vs stream feeds at c2 and c4
# (feed_ms_per_batch = the feeder's per-stage host times), and a c5 kernel trace for k_adam_sumsq.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_autograph.py \
  tests/test_gpu_parity.py -k "autograph or adam" > gpurun_out/r3_feed_tests.log 2>&1 \
  || { tail -60 gpurun_out/r3_feed_tests.log; exit 1; }
tail -3 gpurun_out/r3_feed_tests.log
for c in c2 c4; do
  for f in resident native stream; do
    timeout -k 10 300 python -u bench.py --config $c --feed $f --steps 60 --warmup 10 --no-cpu-baseline --no-roofline \
      --no-eager > gpurun_out/r3_feed_${c}_${f}.json 2> gpurun_out/r3_feed_${c}_${f}.err || { echo "$c $f failed"; tail -20 gpurun_out/r3_feed_${c}_${f}.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('feed_ms_per_batch'))" gpurun_out/r3_feed_${c}_${f}.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_c5" -o c5 -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-eager \
  > "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_c5.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_c5.log"; exit 1; }
f=$(find "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_c5" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && grep -i "adam\|Name" "$f"
exit 0
