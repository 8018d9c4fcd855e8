"""Per-kernel time of ONE replayed train step from a rocprofv3 kernel trace (between two
consecutive k_embed_gather dispatches, i.e. one forward start to the next)."""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
f = max(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True), key=os.path.getmtime)
tr = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(tr) if "k_embed_gather" in r["Kernel_Name"]]
a, b = starts[-3], starts[-2]
seq = tr[a:b]
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seq) / 1e3
print(f"one step: {len(seq)} kernels, span {span:.1f} us, busy {busy:.1f} us")


def short(n):
    n = n.replace("void ", "").replace("aimx::(anonymous namespace)::", "")
    if n.startswith("at::native"):
        n = re.sub(r"<.*", "", n.replace("at::native::(anonymous namespace)::", "").replace("at::native::", ""))
        return "torch:" + n[:60]
    m = re.match(r"([\w:]+(<[^()]*>)?)", n)
    return m.group(1) if m else n[:60]


c, t = collections.Counter(), collections.Counter()
for r in seq:
    k = short(r["Kernel_Name"])
    c[k] += 1
    t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in sorted(t.items(), key=lambda kv: -kv[1]):
    print(f"{v:8.1f} us {c[k]:4d}  {v / c[k]:6.1f} avg  {k}")
