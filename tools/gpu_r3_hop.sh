#!/bin/bash
# Round 3: the odd-width hop (hop_rows.hip): parity tests, then roofline / in-step A/B over knobs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hop_rows.py \
  tests/test_gpu_parity.py -k "hop or model_case" > gpurun_out/r3_hop_tests.log 2>&1 || { tail -50 gpurun_out/r3_hop_tests.log; exit 1; }
tail -3 gpurun_out/r3_hop_tests.log
out=gpurun_out/r3_hop_ab.jsonl; : > $out
for ev in "" "AIMX_HOPR_SPLIT=0" "AIMX_HOPR_SPLIT=1" "AIMX_HOP_ROWS=0" ${EXTRA_ENVS}; do
  env $ev timeout -k 10 300 python -u tools/hop_cfg_micro.py --configs ${CFGS:-c4,c5} >> $out 2>/dev/null || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r3_hop_ab.jsonl"):
    r = json.loads(l); s = r["in_step"]; f = r.get("roofline", {})
    print(r["config"], f"[{r['env']}]", "step fwd", s["fwd"]["us_per_launch"], "bwd", s["bwd"]["us_per_launch"],
          "| roof fwd", f.get("fwd_frac"), "bwd", f.get("bwd_frac"))
PY
