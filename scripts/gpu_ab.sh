#!/bin/bash
# A/B bench of alternative librq builds / plan knobs.  usage: scripts/gpu_ab.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=${1:-ab}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
cd "$ROOT"
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/b$i.log" 2>&1 || { echo "[$E] failed"; tail -5 "$OUT/b$i.log"; exit 1; }
  python3 -c "import json; l=json.loads(open('$OUT/b$i.log').read().strip().splitlines()[-1]); print('[$E]', round(l['value']), l['kernels_ms_per_launch'], l['sweep_plan'])"
done
