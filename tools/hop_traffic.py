"""Combine two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --roofline-only
[--config cN]` into measured HBM bytes per launch of the hop kernel at roofline size, forward and
backward (told apart by grid size: the forward also covers the zero hop chunks).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half of the bytes of a wide
coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE * 1024 is exact for
16-B-per-lane streaming stores.

usage: python tools/hop_traffic.py <fetch_dir> <write_dir> <roofline_json_log> [out.json]
       [--kernel k_gather_sum|k_gather_unal|k_gather_rows]
"""
import argparse
import csv
import glob
import json
import os


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    return list(csv.DictReader(open(max(files, key=os.path.getmtime))))


def per_grid(rs, counter, kernel):
    """{grid size: (mean counter value per dispatch, dispatches)} of the kernel's dispatches."""
    vals = {}
    for r in rs:
        if kernel not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        key = (r.get("Dispatch_Id"), grid)
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {kernel} {counter} rows")
    out = {}
    for (_, g), v in vals.items():
        s, n = out.get(g, (0.0, 0))
        out[g] = (s + v, n + 1)
    return {g: (s / n, n) for g, (s, n) in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("log")
    ap.add_argument("out", nargs="?", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                           "profiles", "hop_traffic.json"))
    ap.add_argument("--kernel", default="k_gather_sum")
    a = ap.parse_args()
    roof = None
    for line in open(a.log):
        line = line.strip()
        if line.startswith("{") and '"bound"' in line:
            roof = json.loads(line)
    if roof is None:
        raise SystemExit("no roofline JSON line in log")
    f, w = per_grid(rows(a.fetch_dir), "FETCH_SIZE", a.kernel), per_grid(rows(a.write_dir), "WRITE_SIZE", a.kernel)
    grids = sorted(set(f) & set(w), key=lambda g: -(f[g][1] + w[g][1]))[:2]  # the two roofline launches
    grids.sort(reverse=True)  # forward (larger grid) first
    rec = {"kernel": a.kernel, "atoms": roof["atoms"], "edges": roof["edges"], "D": roof["D"], "hops": roof["hops"],
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024"}
    algs = [roof["algorithmic_bytes_per_launch"], (roof.get("bwd") or {}).get("algorithmic_bytes_per_launch")]
    for name, g, alg in zip(("fwd", "bwd"), grids, algs):
        part = {"grid": g, "dispatches_averaged": [f[g][1], w[g][1]], "fetch_size_kb": f[g][0],
                "write_size_kb": w[g][0], "read_bytes_per_launch": 2 * f[g][0] * 1024,
                "write_bytes_per_launch": w[g][0] * 1024}
        part["hbm_bytes_per_launch"] = part["read_bytes_per_launch"] + part["write_bytes_per_launch"]
        if alg:
            part["algorithmic_bytes_per_launch"] = alg
            part["traffic_over_algorithmic"] = part["hbm_bytes_per_launch"] / alg
        if name == "fwd":
            rec.update(part)  # the forward's figures at the top level (bench.py reads these)
        else:
            rec["bwd"] = part
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
