#!/bin/bash
# Iteration loop on the box: engine parity tests, the C3 bench line, and (when the
# diagnostic build exists) the per-phase clock split.  usage: scripts/gpu_quick.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-q}
K=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
else
  timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
fi
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
python3 -c "import json; l=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print('C3', round(l['value']), 'replicas/s', round(l['ms_per_step'],3), 'ms/step', l['kernels_ms_per_launch'])"
if [ -f redqueen_amd/librq_clk.so ]; then
  RQ_SO_PATH=$ROOT/redqueen_amd/librq_clk.so timeout -k 10 200 python3 scripts/phase_clock.py > "$OUT/clk.log" 2>&1 || { echo "clk failed"; tail -5 "$OUT/clk.log"; exit 1; }
  tail -2 "$OUT/clk.log"
fi
