#!/bin/bash
# Round 3: k_gather_rows with next-pass staging prefetch (AIMX_HOPR_PREFETCH): bit-exact tests, then the
# roofline / in-step A/B at c4 / c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3_pre; mkdir -p $O
AIMX_HOPR_PREFETCH=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hop_rows.py \
  tests/test_gpu_parity.py -k "hop or model_case" > $O/tests.log 2>&1 || { tail -50 $O/tests.log; exit 1; }
tail -3 $O/tests.log
out=$O/ab.jsonl; : > $out
for ev in "AIMX_HOPR_PREFETCH=1" "AIMX_HOPR_PREFETCH=0" "AIMX_HOPR_PREFETCH=1"; do
  env $ev timeout -k 10 300 python -u tools/hop_cfg_micro.py --configs c4,c5 >> $out 2>/dev/null || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r3_pre/ab.jsonl"):
    r = json.loads(l); s = r["in_step"]; f = r.get("roofline", {})
    print(r["config"], f"[{r['env']}]", "step fwd", s["fwd"]["us_per_launch"], "bwd", s["bwd"]["us_per_launch"],
          "| roof fwd", f.get("fwd_frac"), "bwd", f.get("bwd_frac"))
PY
