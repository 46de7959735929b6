#!/bin/bash
# one --pmc pass over a short bench run; prints the sweep/scan/gen counter values
# usage: scripts/pmc_one.sh WORKLOAD REPLICAS COUNTER [COUNTER...]
set -o pipefail
WL=$1; R=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc1_${WL}_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT" -o p -- python3 bench.py --workload $WL --replicas $R --steps 1 --warmup 1 --no-cpu > "$OUT/log" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][:60]
    acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    if any(x in k for x in ("rq_sweep", "rq_scan", "rq_gen")):
        print("%-60s %-14s %.4g (mean of %d)" % (k, c, sum(v) / len(v), len(v)))
PY
