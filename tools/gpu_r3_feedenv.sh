#!/bin/bash
# Round 3: c2 stream feed throughput alone under page-fault knobs (file pre-mapping, malloc
# thresholds that keep the chunk stores off fresh mmaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_feedenv; mkdir -p $O
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 300 python -u tools/feed_rate.py --config c2 --feed stream --threads 4 --read-threads 12 > $O/$l.json 2> $O/$l.err \
    || { echo "$l failed"; tail -20 $O/$l.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_batch'], d['stages'])" $O/$l.json $l
}
run base A=1
run populate AIMX_H5_POPULATE=1
run malloc GLIBC_TUNABLES=glibc.malloc.mmap_threshold=33554432:glibc.malloc.trim_threshold=4294967296
run both AIMX_H5_POPULATE=1 GLIBC_TUNABLES=glibc.malloc.mmap_threshold=33554432:glibc.malloc.trim_threshold=4294967296
run base2 A=1
rm -f /tmp/aimx_stream_*.h5
exit 0
