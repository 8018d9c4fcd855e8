"""ms_per_step of the last JSON line of each bench log given (gpurun_out/...): one line per file."""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [x for x in open(f) if x.startswith("{")][-1]
        d = json.loads(line)
        print(f"{f}: {d['ms_per_step']} ms/step  value {d['value']}  eager {d.get('eager', {}).get('ms_per_step')}")
    except (OSError, IndexError, ValueError) as e:
        print(f"{f}: no bench line ({type(e).__name__})")
