#!/bin/bash
# merge walk rework: clock split, C5 bench, C5 phase skips, parity tests
set -o pipefail
TAG=${1:-m3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
RQ_SO_PATH=$ROOT/redqueen_amd/librq_mclk.so timeout -k 10 200 python3 -u scripts/dev/merge_clock.py > "$OUT/clock.log" 2>&1 || { echo "clock failed"; tail -5 "$OUT/clock.log"; exit 1; }
grep -v amdgpu.ids "$OUT/clock.log"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_engine.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
scripts/dev/gpu_dbg_c5.sh ${TAG}_dbg || exit 1
