#!/bin/bash
# merged fused sweep: waves per SIMD 4 (default build) / 5 / 6 on C3
set -o pipefail
TAG=${1:-wpe}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
SO=$ROOT/redqueen_amd
b() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); p=d['sweep_plan']; print('$n', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_launch'].items()}, p['waves_per_block'], p['blocks_per_cu'])"
}
b w4 RQ_X=0 || exit 1
b w5 RQ_SO_PATH=$SO/librq_fwm5.so || exit 1
b w6 RQ_SO_PATH=$SO/librq_fwm6.so || exit 1
b w4b RQ_X=0 || exit 1
b w5b RQ_SO_PATH=$SO/librq_fwm5.so || exit 1
