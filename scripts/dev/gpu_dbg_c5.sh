#!/bin/bash
# C5 sweep phase skips (RQ_SWEEP_DBG: 1 skip phase C, 2 skip the sink updates, 3 skip the
# controller) on the merged path.  Output: gpurun_out/$TAG.
set -o pipefail
TAG=${1:-dbg}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for d in 0 1 2 3; do
  RQ_SWEEP_DBG=$d timeout -k 10 200 python3 -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu > "$OUT/d$d.json" 2>"$OUT/d$d.err" || { echo "d$d failed"; tail -5 "$OUT/d$d.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/d$d.json')); print('dbg $d', {k: round(v,2) for k,v in d['kernels_ms_per_launch'].items()})"
done
