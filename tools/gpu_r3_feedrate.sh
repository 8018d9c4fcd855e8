#!/bin/bash
# Round 3: feeder throughput alone (no step) at c2 / c4, native and stream, 8 / 12 threads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_feedrate; mkdir -p $O
ulimit -u; cat /sys/fs/cgroup/pids.max /sys/fs/cgroup/pids.current 2>/dev/null; ps -eLf | wc -l
for c in c2 c4; do
  for f in native stream; do
    for t in 8 12; do
      timeout -k 10 300 python -u tools/feed_rate.py --config $c --feed $f --threads $t >> $O/rate.jsonl 2> $O/${c}_${f}_${t}.err \
        || { echo "$c $f $t failed"; tail -20 $O/${c}_${f}_${t}.err; exit 1; }
      tail -1 $O/rate.jsonl
    done
  done
done
rm -f /tmp/aimx_stream_*.h5
exit 0
