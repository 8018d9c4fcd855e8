#!/bin/bash
# Round 3: Adam fold split (tests + c5 kernel times), feed stage times at c2 / c4, and a c4
# native-feed trace (kernels + memory copies) to see where the fed step loses time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_feed3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_feed.py \
  tests/test_gpu_parity.py tests/test_gpu_train.py -k "feed or feeder or adam or train" > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in c2 c4; do
  for f in native stream; do
    timeout -k 10 400 python -u bench.py --config $c --feed $f --steps 200 --warmup 20 --no-cpu-baseline --no-roofline \
      --no-eager > $O/${c}_${f}.json 2> $O/${c}_${f}.err || { echo "$c $f failed"; tail -20 $O/${c}_${f}.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('feed_ms_per_batch'))" $O/${c}_${f}.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$GRAFT_REPO_ROOT/$O/prof_c4n" -o c4n -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --feed native --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-eager \
  > "$GRAFT_REPO_ROOT/$O/prof_c4n.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/prof_c4n.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/prof_c5" -o c5 -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-eager \
  > "$GRAFT_REPO_ROOT/$O/prof_c5.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/prof_c5.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
db=$(find $O/prof_c5 -name "*.db" | head -1)
python tools/rocpd_summary.py "$db" --top 40 > $O/prof_c5_summary.txt && grep -i "adam\|dispatches" $O/prof_c5_summary.txt
db=$(find $O/prof_c4n -name "*.db" | head -1)
python tools/rocpd_summary.py "$db" --top 40 > $O/prof_c4n_summary.txt && grep -i "copy\|blit\|dispatches" $O/prof_c4n_summary.txt | head
rm -f /tmp/aimx_stream_*.h5
exit 0
