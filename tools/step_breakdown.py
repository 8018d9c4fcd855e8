"""Per-step kernel time of bench.py from a rocprofv3 kernel_trace.csv (steps delimited by the
three CSR builds each forward performs). usage: step_breakdown.py trace.csv [skip_steps]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [i for i, r in enumerate(rows) if "k_count" in r["Kernel_Name"]]
starts = ks[::3]
s0, s1 = starts[skip], starts[-1]
n = len(starts) - 1 - skip
seg = rows[s0:s1]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[s1]["Start_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"per step: wall {(t1 - t0) / n / 1e3:.1f} us, kernels busy {busy / n / 1e3:.1f} us, "
      f"{len(seg) / n:.1f} dispatches")
agg = defaultdict(lambda: [0, 0])
for r in seg:
    nm = r["Kernel_Name"]
    m = re.search(r"aimx::\(anonymous namespace\)::(\w+)(<[^(]*>)?", nm)
    if m:
        key = m.group(1) + (m.group(2) or "")
        if "k_gemm" in key:
            key += f" grid={int(r['Grid_Size_X']) // 256}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    else:
        key = "[torch/rt] " + nm.split("(")[0].replace("void ", "")[-60:]
    agg[key][0] += 1
    agg[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{d / n / 1e3:8.1f} us/step {c / n:5.1f}x avg {d / c / 1e3:6.1f} us  {k}")
