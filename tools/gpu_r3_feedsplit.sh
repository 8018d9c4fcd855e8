#!/bin/bash
# Round 3: c2 stream feed throughput alone, collate threads x reader threads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_feedsplit; mkdir -p $O
for tr in "8 8" "4 8" "4 12" "6 10" "8 12" "2 12" "4 16"; do
  set -- $tr
  timeout -k 10 300 python -u tools/feed_rate.py --config c2 --feed stream --threads $1 --read-threads $2 >> $O/rate.jsonl 2> $O/e_$1_$2.err \
    || { echo "$1 $2 failed"; tail -20 $O/e_$1_$2.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['threads'], d['read_threads'], d['ms_per_batch'], d['stages'])" $O/rate.jsonl
done
rm -f /tmp/aimx_stream_*.h5
exit 0
