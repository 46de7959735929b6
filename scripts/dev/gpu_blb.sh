#!/bin/bash
# BL batch width of the merged-stream sweep (RQ_MRG_BLB 4 default, 2, 8) on C5, plus the
# sweep's FETCH/WRITE bytes for the default build.  Output: gpurun_out/$TAG.
set -o pipefail
TAG=${1:-blb}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
SO=$ROOT/redqueen_amd
b() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernels_ms_per_launch'].items()})"
}
b blb4 RQ_X=0 || exit 1
b blb2 RQ_SO_PATH=$SO/librq_blb2.so || exit 1
b blb8 RQ_SO_PATH=$SO/librq_blb8.so || exit 1
b blb4b RQ_X=0 || exit 1
B="bench.py --steps 2 --warmup 1 --no-cpu --workload c5"
timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/p3" -o p3 -- python3 $B > "$OUT/p3.log" 2>&1 || { echo p3 failed; tail -5 "$OUT/p3.log"; exit 1; }
timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/p4" -o p4 -- python3 $B > "$OUT/p4.log" 2>&1 || { echo p4 failed; tail -5 "$OUT/p4.log"; exit 1; }
python3 scripts/pmc_summary.py "$OUT" workload=c5 | grep -E "^rq_" | cut -c1-400
