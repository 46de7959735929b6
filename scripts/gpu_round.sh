#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, kernel-trace profile.  usage: scripts/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
echo "pytest ok"; tail -3 "$OUT/pytest.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/kt.log" 2>&1 || { echo "rocprof failed"; tail -30 "$OUT/kt.log"; exit 1; }
tail -1 "$OUT/kt.log"
find "$OUT/kt" -name "*kernel_stats.csv" -exec cat {} \;
