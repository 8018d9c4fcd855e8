#!/bin/bash
# Round 3: two ranks sharing the box's GPU over gloo (rehearsal of the data-parallel feed paths:
# stream shards, static capacity, replica check), then the step kernel sequences.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_rehearse; mkdir -p $O
for spec in "c4 stream" "c2 native"; do
  set -- $spec
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --dist-backend gloo --config $1 --feed $2 --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --no-eager \
    > $O/$1_$2.json 2> $O/$1_$2.err || { echo "$1 $2 rc=$?"; tail -30 $O/$1_$2.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d.get('ddp'), d.get('graph_eager_steps'), d.get('feed_ms_per_batch'))" $O/$1_$2.json
done
rm -f /tmp/aimx_stream_*.h5
bash tools/gpu_seq.sh || exit 1
exit 0
