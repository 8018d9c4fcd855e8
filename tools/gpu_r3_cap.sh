#!/bin/bash
# Round 3: static capacity from max + 1 sd (over-capacity batches stepped eagerly): feed / train
# tests, then c2 / c4 stream and native feeds against resident.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_cap; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_feed.py tests/test_gpu_train.py \
  tests/test_gpu_ddp.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in c2 c4; do
  for f in resident native stream; do
    timeout -k 10 400 python -u bench.py --config $c --feed $f --steps 300 --warmup 20 --no-cpu-baseline --no-roofline \
      --no-eager > $O/${c}_${f}.json 2> $O/${c}_${f}.err || { echo "$c $f failed"; tail -20 $O/${c}_${f}.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('graph_eager_steps'), d.get('feed_ms_per_batch'), d['config'].get('mean_atoms_per_batch'))" $O/${c}_${f}.json
  done
done
rm -f /tmp/aimx_stream_*.h5
exit 0
