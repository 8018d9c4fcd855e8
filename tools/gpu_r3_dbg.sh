#!/bin/bash
# Round 3: phase knock-out timing of hop_rows.hip (AIMX_HOPR_DBG bits; results wrong by design).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
out=gpurun_out/r3_hopr_dbg.jsonl; : > $out
for dbg in 0 1 2 4 8 3 7 15; do
  AIMX_HOPR_DBG=$dbg timeout -k 10 120 python -u tools/hop_cfg_micro.py --configs c4,c5 --no-roofline >> $out 2>/dev/null || exit 1
done
for w in 16 64 128; do
  AIMX_HOPR_WIN=$w timeout -k 10 120 python -u tools/hop_cfg_micro.py --configs c5 --no-roofline >> $out 2>/dev/null || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r3_hopr_dbg.jsonl"):
    r = json.loads(l); s = r["in_step"]
    print(r["config"], r["env"], "fwd", s["fwd"]["us_per_launch"], "bwd", s["bwd"]["us_per_launch"])
PY
