"""One line per bench_paths.py result file: (ms, GB/s, equal to the sweep) per section."""
import json
import sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = d.get("sections", d)
out = {}
for k, v in d.items():
    if isinstance(v, dict):
        ms = v.get("ms_fast", v.get("ms_replay", v.get("ms")))
        if ms is not None:
            out[k] = (round(ms, 3), round(v.get("GBps", 0)), v.get("equal_to_sweep"))
print(sys.argv[2], out)
