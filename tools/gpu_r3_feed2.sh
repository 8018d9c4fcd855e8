#!/bin/bash
# Round 3: feed ring + parallel collate CSR + direct HDF5 reads: GPU feed tests, resident vs
# native vs stream at c2 / c4 (timed-region feed stage times), and a 1M-molecule c4 stream file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_feed2; mkdir -p $O
df -h /tmp "${TMPDIR:-/tmp}" | tail -2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_feed.py \
  tests/test_gpu_autograph.py tests/test_gpu_parity.py -k "feed or feeder or autograph or adam" > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in c2 c4; do
  for f in resident native stream; do
    timeout -k 10 400 python -u bench.py --config $c --feed $f --steps 200 --warmup 20 --no-cpu-baseline --no-roofline \
      --no-eager > $O/${c}_${f}.json 2> $O/${c}_${f}.err || { echo "$c $f failed"; tail -20 $O/${c}_${f}.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('feed_ms_per_batch'), d.get('stream_file'))" $O/${c}_${f}.json
  done
done
timeout -k 10 900 python -u bench.py --config c4 --feed stream --stream-mols 1000000 --steps 300 --warmup 20 \
  --no-cpu-baseline --no-roofline --no-eager > $O/c4_stream_1M.json 2> $O/c4_stream_1M.err || { echo "1M failed"; tail -20 $O/c4_stream_1M.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('feed_ms_per_batch'), d.get('stream_file'))" $O/c4_stream_1M.json

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/prof_c5" -o c5 -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-eager \
  > "$GRAFT_REPO_ROOT/$O/prof_c5.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/prof_c5.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
db=$(find $O/prof_c5 -name "*.db" | head -1)
python tools/rocpd_summary.py "$db" --top 40 > $O/prof_c5_summary.txt && grep -i "adam\|dispatches" $O/prof_c5_summary.txt
rm -f /tmp/aimx_stream_*.h5
