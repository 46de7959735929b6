#!/bin/bash
# A/B of environment knobs on the C3 bench (and the phase clock of the diagnostic
# build).  usage: scripts/gpu_envab.sh TAG "ENV1" "ENV2" ...   e.g. "RQ_FW_W=16" "RQ_FW_W=32"
set -o pipefail
TAG=${1:-ab}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/bench$i.log" 2>&1 || { echo "bench $E failed"; tail -5 "$OUT/bench$i.log"; exit 1; }
  python3 -c "import json; l=json.loads(open('$OUT/bench$i.log').read().strip().splitlines()[-1]); print('$E', round(l['value']), 'replicas/s', round(l['ms_per_step'],3), 'ms/step', l['kernels_ms_per_launch']['sweep'], l['sweep_plan'])"
  if [ -f redqueen_amd/librq_clk.so ]; then
    env $E RQ_SO_PATH=$ROOT/redqueen_amd/librq_clk.so timeout -k 10 200 python3 scripts/phase_clock.py > "$OUT/clk$i.log" 2>&1 || { echo "clk failed"; tail -5 "$OUT/clk$i.log"; exit 1; }
    tail -2 "$OUT/clk$i.log"
  fi
done
