"""Per-kernel MFMA utilisation from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE (one row per dispatch and counter).

MfmaUtil follows rocprofv3's own derived counter (counters list, `rocprofv3 -L`):
  sum(SQ_VALU_MFMA_BUSY_CYCLES) / (max GRBM_GUI_ACTIVE * SIMD_NUM) * 100
rocprofv3 reports GRBM_GUI_ACTIVE summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS notes), so the
per-XCD max is taken as sum / 8; SIMD_NUM = 256 CUs x 4 SIMDs. Aggregated per kernel name as
busy-weighted means (sum of MFMA cycles / sum of available SIMD-cycles).

usage: python tools/mfma_summary.py <pmc dir> [top]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMD_NUM = 256 * 4
XCD = 8


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    path = max(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True), key=os.path.getmtime)
    per = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for k, c in per.items():
        if "GRBM_GUI_ACTIVE" not in c:
            continue
        n = names[k].replace("aimx::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        a = agg[n]
        a[0] += 1
        a[1] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a[2] += c["GRBM_GUI_ACTIVE"] / XCD * SIMD_NUM
    tot_b = sum(a[1] for a in agg.values())
    tot_t = sum(a[2] for a in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][2])
    out = {"all_kernels_mfma_util_pct": round(100 * tot_b / tot_t, 2), "kernels": []}
    for n, (cnt, b, t) in rows[:top]:
        out["kernels"].append({"kernel": n, "dispatches": cnt, "share_of_gpu_time_pct": round(100 * t / tot_t, 2),
                               "mfma_util_pct": round(100 * b / t, 2)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
