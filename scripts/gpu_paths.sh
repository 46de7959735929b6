#!/bin/bash
# bench_paths.py + its kernel trace + FETCH/WRITE passes.  usage: scripts/gpu_paths.sh TAG
set -o pipefail
TAG=${1:-paths}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python3 scripts/bench_paths.py > "$OUT/paths.json" 2> "$OUT/paths.err" || { echo paths failed; tail -20 "$OUT/paths.err"; exit 1; }
cat "$OUT/paths.json"
P="--output-format csv"
timeout -k 10 300 rocprofv3 --kernel-trace --stats $P -d "$OUT/kt" -o kt -- python3 scripts/bench_paths.py --reps 1 > "$OUT/kt.log" 2>&1 || { echo kt failed; tail -5 "$OUT/kt.log"; exit 1; }
echo kt ok
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE $P -d "$OUT/p3" -o p3 -- python3 scripts/bench_paths.py --reps 1 > "$OUT/p3.log" 2>&1 || { echo p3 failed; tail -5 "$OUT/p3.log"; exit 1; }
echo fetch ok
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE $P -d "$OUT/p4" -o p4 -- python3 scripts/bench_paths.py --reps 1 > "$OUT/p4.log" 2>&1 || { echo p4 failed; tail -5 "$OUT/p4.log"; exit 1; }
echo write ok
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.txt"
grep -v "^ " "$OUT/summary.txt"
