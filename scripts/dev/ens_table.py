"""Markdown table of ensemble comparisons from RQ_ENSEMBLE_LOG JSON lines (tests/ensemble.py)."""
import json
import sys

rows = {}
for path in sys.argv[1:]:
    for line in open(path):
        line = line.strip()
        if line:
            d = json.loads(line)
            rows[d["name"]] = d
print("| comparison | engine / reference replicas | statistics | max abs z (bound) | smallest p: spread / shape (bound) |")
print("|---|---|---|---|---|")
for name in sorted(rows):
    d = rows[name]
    print("| `%s` | %d / %d | %d | %.2f (%.2f) | %.3g / %.3g (%.2g) |" % (
        name, d["n_eng"], d["n_ref"], len(d["stats"]), d["max_abs_z"], d["z_bound"],
        d["min_p_spread"], d["min_p_shape"], d["p_bound"]))
