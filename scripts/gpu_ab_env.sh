#!/bin/bash
# A/B of library env knobs on one box: the GPU suite (optional), then bench.py lines
# for each "NAME=ENV..." variant.  usage:
#   scripts/gpu_ab_env.sh TAG [--tests] [--workload c3] [--steps 20] -- "base=" "p1=RQ_PIPE=1" ...
set -o pipefail
TAG=$1; shift
TESTS=0; WL=c3; STEPS=20
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case "$1" in
    --tests) TESTS=1 ;;
    --workload) WL=$2; shift ;;
    --steps) STEPS=$2; shift ;;
  esac
  shift
done
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
if [ "$TESTS" = 1 ]; then
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
for v in "$@"; do
  name=${v%%=*}; envs=${v#*=}
  env $envs timeout -k 10 300 python3 -u bench.py --workload "$WL" --steps "$STEPS" --warmup 3 --no-cpu > "$OUT/bench_$name.log" 2>&1 || { echo "bench $name failed"; tail -5 "$OUT/bench_$name.log"; exit 1; }
  python3 -c "import json,sys; l=json.loads(open('$OUT/bench_$name.log').read().strip().splitlines()[-1]); print('$name', '$envs', round(l['value']), 'replicas/s', round(l['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()}, 'plan chunk', l['sweep_plan']['chunk'], 'sweep alone', l['roofline'].get('duration_ms'), 'frac', l['roofline'].get('frac'))"
done
