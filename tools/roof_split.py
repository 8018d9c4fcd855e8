"""Split a `rocprofv3 --kernel-trace` CSV of `bench.py --roofline-only` into the hop's forward and
backward launches (the same kernel name; the forward's grid also covers the zero hop chunks, so
it is the larger one) and report each one's average device duration next to the bench's HIP-event
figures and algorithmic bytes.

usage: python tools/roof_split.py <trace dir> <roofline log (bench JSON line)> [out.json]
"""
import csv
import glob
import json
import os
import sys


def main():
    d, log = sys.argv[1:3]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    path = max(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True), key=os.path.getmtime)
    roof = [json.loads(l) for l in open(log) if l.startswith("{") and '"bound"' in l][-1]
    kname = roof["kernel"].split()[0]
    groups = {}
    for r in csv.DictReader(open(path)):
        if kname not in r["Kernel_Name"]:
            continue
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        groups.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    big = sorted(groups, key=lambda g: -len(groups[g]))[:2]
    big.sort(reverse=True)
    rec = {"kernel": kname, "atoms": roof["atoms"], "edges": roof["edges"], "D": roof["D"], "hops": roof["hops"]}
    for name, g, alg, ev_us in zip(("fwd", "bwd"), big,
                                   (roof["algorithmic_bytes_per_launch"], roof["bwd"]["algorithmic_bytes"]),
                                   (roof["ms_per_launch"] * 1e3, roof["bwd"]["us_per_launch"])):
        ds = groups[g]
        avg = sum(ds) / len(ds)
        rec[name] = {"grid": g, "launches": len(ds), "rocprof_avg_us": round(avg, 2), "hip_event_us": round(ev_us, 2),
                     "algorithmic_bytes": alg, "achieved_GBs_rocprof": round(alg / avg / 1e3, 1),
                     "frac_of_8TBs_rocprof": round(alg / avg / 1e3 / 8000.0, 4)}
    print(json.dumps(rec))
    if out:
        json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
