"""Per-step kernel breakdown from a rocprofv3 kernel_trace.csv of bench.py.

Finds the training-step window (before the first hop-roofline launch, i.e. the first
k_gather_sum longer than 500 us), splits it into `steps` equal parts by dispatch count of the
step-marker kernel, and prints per-step time by kernel plus per-GEMM-shape detail.
usage: python tools/trace_summary.py <kernel_trace.csv> <num_steps_total>
"""
import csv
import sys
from collections import defaultdict


def main(path, nsteps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # cut at the roofline: first long gather
    cut = len(rows)
    for i, r in enumerate(rows):
        if "k_gather_sum" in r["Kernel_Name"] and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 500_000:
            cut = i
            break
    rows = rows[:cut]
    # drop the data-prep prefix: start at the first k_count (CSR build of step 0)
    first = next(i for i, r in enumerate(rows) if "k_count" in r["Kernel_Name"])
    rows = rows[first:]
    t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
    agg = defaultdict(lambda: [0, 0.0])
    shapes = defaultdict(lambda: [0, 0.0])
    busy = 0
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "")[-60:]
        agg[short][0] += 1
        agg[short][1] += d
        if "k_gemm" in name or "Cijk" in name:
            key = (short[-30:], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
            shapes[key][0] += 1
            shapes[key][1] += d
    print(f"window {(t1 - t0) / 1e3 / nsteps:.1f} us/step wall, kernels busy {busy / nsteps:.1f} us/step, "
          f"{len(rows) / nsteps:.1f} dispatches/step")
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {d / nsteps:8.1f} us/step  {c / nsteps:5.1f}x  {k}")
    print("GEMM shapes (grid x,y,z):")
    for k, (c, d) in sorted(shapes.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"  {d / nsteps:8.1f} us/step  {c / nsteps:5.1f}x  avg {d / c:7.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
