#!/bin/bash
# C5 evidence: bench.py --workload c5 + its rocprofv3 kernel stats; C3 bench for comparison.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
R=${C5_REPLICAS:-2560}
timeout -k 10 300 python3 -u bench.py --workload c5 --replicas $R --steps 3 --warmup 1 --no-cpu > "$OUT/c5_bench.log" 2>&1 || { echo c5 bench failed; tail -20 "$OUT/c5_bench.log"; exit 1; }
tail -1 "$OUT/c5_bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py --workload c5 --replicas $R --steps 3 --warmup 1 --no-cpu > "$OUT/kt.log" 2>&1 || { echo kt failed; tail -5 "$OUT/kt.log"; exit 1; }
find "$OUT/kt" -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/c3_bench.log" 2>&1 || { echo c3 bench failed; exit 1; }
tail -1 "$OUT/c3_bench.log" | cut -c1-400
