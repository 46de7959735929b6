#!/bin/bash
# C3 merge phase clock + C3 bench + merge tests
set -o pipefail
TAG=${1:-m4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
RQ_WL=c3 RQ_SO_PATH=$ROOT/redqueen_amd/librq_mclk.so timeout -k 10 200 python3 -u scripts/dev/merge_clock.py > "$OUT/clock.log" 2>&1 || { echo "clock failed"; tail -5 "$OUT/clock.log"; exit 1; }
grep -v amdgpu.ids "$OUT/clock.log"
for n in a b; do
  timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_launch'].items()})"
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
