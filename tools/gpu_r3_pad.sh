#!/bin/bash
# Round 3: padding molecules of <= 64 atoms (feeds, resident pool, autograph buckets): tests,
# fed vs resident at c2 / c4, and eager vs autograph (default gate and forced) at c2-c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_pad; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_feed.py \
  tests/test_gpu_autograph.py tests/test_gpu_train.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d.get('eager') or {}; print(sys.argv[2], d['ms_per_step'], 'eager', e.get('ms_per_step'), 'autograph', (e.get('autograph') or {}).get('ms_per_step'), d.get('feed_ms_per_batch'))" "$@"; }
for c in c2 c4; do
  for f in resident native stream; do
    timeout -k 10 400 python -u bench.py --config $c --feed $f --steps 200 --warmup 20 --no-cpu-baseline --no-roofline \
      --no-eager > $O/${c}_${f}.json 2> $O/${c}_${f}.err || { echo "$c $f failed"; tail -20 $O/${c}_${f}.err; exit 1; }
    show $O/${c}_${f}.json "$c $f"
  done
done
for c in c2 c3 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 30 --warmup 10 --no-cpu-baseline --no-roofline \
    > $O/${c}_eager.json 2> $O/${c}_eager.err || { echo "$c eager failed"; tail -20 $O/${c}_eager.err; exit 1; }
  show $O/${c}_eager.json "$c default"
  AIMX_AUTOGRAPH_MAX_WORK=1e12 timeout -k 10 400 python -u bench.py --config $c --steps 30 --warmup 10 --no-cpu-baseline \
    --no-roofline > $O/${c}_eagerf.json 2> $O/${c}_eagerf.err || { echo "$c forced failed"; tail -20 $O/${c}_eagerf.err; exit 1; }
  show $O/${c}_eagerf.json "$c forced-autograph"
done
rm -f /tmp/aimx_stream_*.h5
