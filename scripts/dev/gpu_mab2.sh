#!/bin/bash
# A/B round 2: merge phase clock, sweep launch bound 768 vs 1024, C3 bench (uniform wave
# index in the fused sweep), engine parity tests.  Output: gpurun_out/$TAG.
set -o pipefail
TAG=${1:-mab2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
SO=$ROOT/redqueen_amd
RQ_SO_PATH=$SO/librq_mclk.so timeout -k 10 200 python3 -u scripts/dev/merge_clock.py > "$OUT/clock.log" 2>&1 || { echo "clock failed"; tail -5 "$OUT/clock.log"; exit 1; }
grep -v amdgpu.ids "$OUT/clock.log"
b() {   # name, workload, env...
  local n=$1 wl=$2; shift 2
  env "$@" timeout -k 10 200 python3 -u bench.py --workload $wl --steps 5 --warmup 1 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_launch'].items()}, d['sweep_plan']['waves_per_block'], d['sweep_plan']['blocks_per_cu'])"
}
b c5base c5 RQ_X=0 || exit 1
b c5lb768 c5 RQ_SO_PATH=$SO/librq_lb768.so || exit 1
b c5base2 c5 RQ_X=0 || exit 1
b c3 c3 RQ_X=0 || exit 1
b c3b c3 RQ_X=0 || exit 1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_merge.py tests/test_gpu_policy.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
