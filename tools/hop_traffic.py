"""Combine two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --roofline-only` into
profiles/hop_traffic.json: measured HBM bytes per launch of the hop kernel at roofline size.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half of the bytes of a wide
coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE * 1024 is exact for
16-B-per-lane streaming stores. Only the largest-grid k_gather_sum dispatches (the roofline
launches, not the CSR build or warm-up of smaller graphs) are averaged.

usage: python tools/hop_traffic.py <fetch_dir> <write_dir> <roofline_json_log> [out.json]
"""
import csv
import glob
import json
import os
import sys


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    # the newest run only (gpurun_out/ keeps the run directories of earlier calls)
    return list(csv.DictReader(open(max(files, key=os.path.getmtime))))


def per_dispatch(rs, counter):
    vals = {}
    for r in rs:
        if "k_gather_sum" not in r.get("Kernel_Name", ""):
            continue
        if r.get("Counter_Name") != counter:
            continue
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        key = (r.get("Dispatch_Id"), grid)
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no k_gather_sum {counter} rows")
    gmax = max(g for _, g in vals)
    sel = [v for (d, g), v in vals.items() if g == gmax]
    return sum(sel) / len(sel), len(sel), gmax


def main():
    fetch_dir, write_dir, log = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "hop_traffic.json")
    f, nf, gf = per_dispatch(rows(fetch_dir), "FETCH_SIZE")
    w, nw, gw = per_dispatch(rows(write_dir), "WRITE_SIZE")
    roof = None
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"bound"' in line:
            roof = json.loads(line)
    if roof is None:
        raise SystemExit("no roofline JSON line in log")
    rec = {
        "kernel": roof["kernel"], "atoms": roof["atoms"], "edges": roof["edges"], "D": roof["D"],
        "hops": roof["hops"], "dispatches_averaged": [nf, nw], "grid": gf,
        "fetch_size_kb": f, "write_size_kb": w,
        "read_bytes_per_launch": 2 * f * 1024, "write_bytes_per_launch": w * 1024,
        "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
        "algorithmic_bytes_per_launch": roof["algorithmic_bytes_per_launch"],
        "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024",
    }
    rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / rec["algorithmic_bytes_per_launch"]
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
