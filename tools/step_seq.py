"""One replayed train step's kernel sequence from a rocprofv3 kernel trace: duration, gap to the
previous kernel, workgroups, name (between two consecutive k_embed_gather dispatches).

usage: python tools/step_seq.py <trace dir>
"""
import csv
import glob
import os
import re
import sys

f = max(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True), key=os.path.getmtime)
tr = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(tr) if "k_embed_gather" in r["Kernel_Name"]]
a, b = starts[-3], starts[-2]
prev = None
tot = 0.0
t_first = int(tr[a]["Start_Timestamp"])
for r in tr[a:b]:
    n = r["Kernel_Name"].replace("void ", "").replace("aimx::(anonymous namespace)::", "")
    if n.startswith("at::native::"):  # keep the kernel and its functor, drop the template noise
        fn = re.findall(r"(\w+(?:Functor|Op|_kernel|Kernel)\w*)", n)
        n = "torch:" + " ".join(dict.fromkeys(fn))[:90]
    else:
        n = re.sub(r"\(.*", "", n)[:70]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    wgs = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]))
    tot += (e - s) / 1e3
    print(f"{(e - s) / 1e3:7.1f} gap {gap:5.1f} at {(s - t_first) / 1e3:7.1f} wgs {wgs:7d}  {n}")
print(f"{b - a} kernels, {tot:.1f} us busy, span {(int(tr[b - 1]['End_Timestamp']) - int(tr[a]['Start_Timestamp'])) / 1e3:.1f} us")
