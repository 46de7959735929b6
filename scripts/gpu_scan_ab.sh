#!/bin/bash
# rq_scan A/B over the waves-per-SIMD builds (RQ_SCAN_WPE) + the full GPU suite.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-scanab}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for w in 4 6 8; do
  RQ_SCAN_WPE=$w timeout -k 10 300 python3 scripts/bench_paths.py --reps 5 > "$OUT/paths_$w.json" 2> "$OUT/paths_$w.err" || { echo "paths $w failed"; tail -5 "$OUT/paths_$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/paths_$w.json')); print('wpe $w scan', d['scan']['ms'], d['scan']['GBps'], 'replay', d['replay_batch']['ms_fast'], d['replay_batch']['ms_scan'], d['replay_batch']['GBps'])"
done
