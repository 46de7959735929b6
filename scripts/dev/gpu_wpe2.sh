#!/bin/bash
# merged fused sweep waves per SIMD (4 / 5 / 6) and the vectorised merge walk (mg0: the
# per-arrival walk) on C3, C5 merge A/B, merge tests
set -o pipefail
TAG=${1:-wpe2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
SO=$ROOT/redqueen_amd
b() {
  local n=$1 wl=$2; shift 2
  env "$@" timeout -k 10 200 python3 -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); p=d['sweep_plan']; print('$n', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_launch'].items()}, p['waves_per_block'], p['blocks_per_cu'])"
}
b w4 c3 RQ_X=0 || exit 1
b mg0 c3 RQ_SO_PATH=$SO/librq_mg0.so || exit 1
b w5 c3 RQ_SO_PATH=$SO/librq_fwm5.so || exit 1
b w6 c3 RQ_SO_PATH=$SO/librq_fwm6.so || exit 1
b w4b c3 RQ_X=0 || exit 1
b c5 c5 RQ_X=0 || exit 1
b c5mg0 c5 RQ_SO_PATH=$SO/librq_mg0.so || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
