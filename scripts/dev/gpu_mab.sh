#!/bin/bash
# A/B of the merged-stream C5 path: merge phase clock, prefetch depth, sweep launch bound,
# column placement.  Output: gpurun_out/$TAG.
set -o pipefail
TAG=${1:-mab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
SO=$ROOT/redqueen_amd
RQ_SO_PATH=$SO/librq_mclk.so timeout -k 10 200 python3 -u scripts/dev/merge_clock.py > "$OUT/clock.log" 2>&1 || { echo "clock failed"; tail -5 "$OUT/clock.log"; exit 1; }
cat "$OUT/clock.log"
b() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['ms_per_step'],1), d['kernels_ms_per_launch'], d['sweep_plan']['waves_per_block'], d['sweep_plan']['columns_in_lds'])"
}
b base RQ_X=0 || exit 1
b pf2 RQ_SO_PATH=$SO/librq_pf2.so || exit 1
b lb512 RQ_SO_PATH=$SO/librq_lb512.so || exit 1
b lb512lds RQ_SO_PATH=$SO/librq_lb512.so RQ_G_COLLDS=1 || exit 1
b collds RQ_G_COLLDS=1 || exit 1
b base2 RQ_X=0 || exit 1
