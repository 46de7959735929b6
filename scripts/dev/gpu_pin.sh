#!/bin/bash
# merged sweeps with the next tile pinned before the row stores: C3 / C5 bench, tests
set -o pipefail
TAG=${1:-pin}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
b() {
  local n=$1 wl=$2; shift 2
  env "$@" timeout -k 10 200 python3 -u bench.py --workload $wl --steps 5 --warmup 2 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); p=d['sweep_plan']; print('$n', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_launch'].items()})"
}
b c3 c3 RQ_X=0 || exit 1
b c3b c3 RQ_X=0 || exit 1
b c5 c5 RQ_X=0 || exit 1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_engine.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
