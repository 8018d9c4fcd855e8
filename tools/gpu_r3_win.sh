#!/bin/bash
# Round 3: windows per workgroup (workgroup count) sweep for hop_rows (c4 / c5) and tile height for
# hop.hip (c2), roofline + in-step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
out=gpurun_out/r3_win.jsonl; : > $out
for ev in "AIMX_X=0" "AIMX_HOPR_WIN=64" "AIMX_HOPR_WIN=128" "AIMX_HOPR_WIN=64 AIMX_HOPR_SPLIT=0" ; do
  env $ev timeout -k 10 300 python -u tools/hop_cfg_micro.py --configs c4,c5 >> $out || exit 1
done
for ev in "AIMX_X=0" "AIMX_HOP_TILE_UNITS=1024" "AIMX_HOP_TILE_UNITS=2048" ; do
  env $ev timeout -k 10 300 python -u tools/hop_cfg_micro.py --configs c2 >> $out || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r3_win.jsonl"):
    r = json.loads(l); s = r["in_step"]; f = r.get("roofline", {})
    print(r["config"], f"[{r['env']}]", "step fwd", s["fwd"]["us_per_launch"], "bwd", s["bwd"]["us_per_launch"],
          "| roof fwd", f.get("fwd_frac"), "bwd", f.get("bwd_frac"))
PY
