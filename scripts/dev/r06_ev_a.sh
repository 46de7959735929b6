#!/bin/bash
# round-6 evidence, part A: the GPU suite, smoke, then the stamped C3 and C4 evidence
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ev06
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --durations=25 --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest.log" | head; tail -3 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
RND=r06 bash scripts/gpu_evidence.sh ev06 "c3 c4"
