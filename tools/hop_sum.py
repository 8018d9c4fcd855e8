"""Summarise tools/hop_cfg_micro.py logs: one line per (log, config)."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        s = f"{f.split('/')[-1]:16s} {d['config']} {d.get('env', '')[:40]:40s}"
        if "in_step" in d:
            i = d["in_step"]
            s += f" in-step fwd {i['fwd']['us_per_launch']:6.1f} bwd {i['bwd']['us_per_launch']:6.1f}"
        if "roofline" in d:
            r = d["roofline"]
            s += f" roof fwd {r['fwd_ms']:.3f} ({r['fwd_frac']:.3f}) bwd {r['bwd_us']:.0f} ({r['bwd_frac']:.3f})"
        print(s)
