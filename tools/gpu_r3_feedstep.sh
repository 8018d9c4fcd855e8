#!/bin/bash
# Round 3: c2 stream feed under the step, stage split (slot wait vs collate), thread splits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_feedstep; mkdir -p $O
for tr in "8 8" "4 12"; do
  set -- $tr
  timeout -k 10 400 python -u bench.py --config c2 --feed stream --feed-threads $1 --read-threads $2 --steps 300 --warmup 20 \
    --no-cpu-baseline --no-roofline --no-eager > $O/c2_$1_$2.json 2> $O/c2_$1_$2.err || { echo "failed"; tail -20 $O/c2_$1_$2.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('feed_ms_per_batch'))" $O/c2_$1_$2.json
done
timeout -k 10 400 python -u bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline --no-roofline --no-eager > $O/c2_res.json 2> $O/c2_res.err || { echo "failed"; tail -20 $O/c2_res.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $O/c2_res.json
rm -f /tmp/aimx_stream_*.h5
exit 0
