#!/bin/bash
# Round 3: hop_rows knob sweep (LDS footprint / window / tile cap) at c4 / c5, roofline + in-step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
out=gpurun_out/r3_knobs.jsonl; : > $out
for ev in "AIMX_X=0" "AIMX_HOPR_COL_CAP=1024" "AIMX_HOPR_CAP=48" "AIMX_HOPR_CAP=48 AIMX_HOPR_COL_CAP=1024" \
          "AIMX_HOPR_WIN=16" "AIMX_HOPR_WIN=64" "AIMX_HOPR_WC=64" "AIMX_HOPR_WC=56" ${EXTRA_ENVS}; do
  env $ev timeout -k 10 300 python -u tools/hop_cfg_micro.py --configs ${CFGS:-c4,c5} >> $out || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r3_knobs.jsonl"):
    r = json.loads(l); s = r["in_step"]; f = r.get("roofline", {})
    print(r["config"], f"[{r['env']}]", "step fwd", s["fwd"]["us_per_launch"], "bwd", s["bwd"]["us_per_launch"],
          "| roof fwd", f.get("fwd_frac"), "bwd", f.get("bwd_frac"))
PY
