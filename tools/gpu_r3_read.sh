#!/bin/bash
# Round 3: HDF5 read rate after file-order decode + in-place store fill, the c2 / c4 stream
# feeds, and the 1M-molecule c4 stream file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_read; mkdir -p $O
df -h /tmp | tail -1; nproc
timeout -k 10 300 python -u tools/h5_read_rate.py --source qm9 --mols 200000 > $O/rate_qm9.txt 2>&1 || { tail -5 $O/rate_qm9.txt; exit 1; }
cat $O/rate_qm9.txt
timeout -k 10 300 python -u tools/h5_read_rate.py --source synth40 --mols 200000 > $O/rate_synth40.txt 2>&1 || { tail -5 $O/rate_synth40.txt; exit 1; }
cat $O/rate_synth40.txt
rm -f /tmp/aimx_rate_*.h5
for c in c2 c4; do
  timeout -k 10 400 python -u bench.py --config $c --feed stream --steps 200 --warmup 20 --no-cpu-baseline --no-roofline \
    --no-eager > $O/${c}_stream.json 2> $O/${c}_stream.err || { echo "$c failed"; tail -20 $O/${c}_stream.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('feed_ms_per_batch'), d.get('stream_file'))" $O/${c}_stream.json
done
rm -f /tmp/aimx_stream_*.h5
timeout -k 10 600 python -u bench.py --config c4 --feed stream --stream-mols 1000000 --steps 400 --warmup 20 --no-cpu-baseline \
  --no-roofline --no-eager > $O/c4_stream_1m.json 2> $O/c4_stream_1m.err || { echo "1m failed"; tail -20 $O/c4_stream_1m.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('feed_ms_per_batch'), d.get('stream_file'))" $O/c4_stream_1m.json
rm -f /tmp/aimx_stream_*.h5
exit 0
