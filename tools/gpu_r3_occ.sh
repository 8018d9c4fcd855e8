#!/bin/bash
# Round 3: hop_rows.hip at the c4 roofline size: occupancy sweep (LDS padding) and phase knock-outs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
out=gpurun_out/r3_occ.jsonl; : > $out
# 26.4 KB per WG: pad 0 -> 6/CU, 8000 -> 4/CU (34 KB), 27000 -> 3/CU (53 KB), 54000 -> 2/CU (80 KB)
for ev in "AIMX_HOPR_LDS_PAD=0" "AIMX_HOPR_LDS_PAD=8000" "AIMX_HOPR_LDS_PAD=27000" "AIMX_HOPR_LDS_PAD=54000" \
          "AIMX_HOPR_DBG=1" "AIMX_HOPR_DBG=2" "AIMX_HOPR_DBG=4" "AIMX_HOPR_DBG=8" "AIMX_HOPR_DBG=3" "AIMX_HOPR_DBG=7" "AIMX_HOPR_DBG=15"; do
  env $ev timeout -k 10 300 python -u tools/hop_cfg_micro.py --configs c4 --no-in-step >> $out 2>/dev/null || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r3_occ.jsonl"):
    r = json.loads(l); f = r["roofline"]
    print(r["config"], f"[{r['env']}]", "fwd ms", f["fwd_ms"], f["fwd_frac"], "bwd us", f["bwd_us"], f["bwd_frac"])
PY
