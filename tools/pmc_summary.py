"""Average every counter of rocprofv3 --pmc output over the largest-grid dispatches of one kernel.

usage: python tools/pmc_summary.py <pmc_dir> [kernel_substring]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 else "k_gather_sum"
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kname not in r.get("Kernel_Name", ""):
                continue
            grid = int(r.get("Grid_Size", 0) or 0)
            key = (r["Counter_Name"], grid)
            vals.setdefault(key, {}).setdefault(r["Dispatch_Id"], 0.0)
            vals[key][r["Dispatch_Id"]] += float(r["Counter_Value"])
    if not vals:
        raise SystemExit("no rows")
    gmax = max(g for _, g in vals)
    for (c, g), per in sorted(vals.items()):
        if g == gmax:
            print(f"{c:40s} {sum(per.values()) / len(per):16.1f}  (n={len(per)}, grid={g})")


if __name__ == "__main__":
    main()
