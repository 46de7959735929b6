#!/bin/bash
# fused sweep on merged streams (C3): bench A/B vs the in-kernel generating sweep
# (RQ_FWM=0), then the engine / merge / policy / config / stats tests
set -o pipefail
TAG=${1:-fwm}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 250 python3 -u scripts/dev/c3_modes2.py > "$OUT/modes.log" 2>&1 || { echo "modes failed"; tail -5 "$OUT/modes.log"; exit 1; }
cat "$OUT/modes.log" | grep -v amdgpu.ids
b() {
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/$n.json" 2>"$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms_per_launch'].items()})"
}
b fwm RQ_X=0 || exit 1
b gen RQ_FWM=0 || exit 1
b fwm2 RQ_X=0 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_merge.py tests/test_gpu_policy.py tests/test_gpu_configs.py tests/test_gpu_stats.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
