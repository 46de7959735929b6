#!/bin/bash
# replay small-table tier: A/B (RQ_RP_SMALL=0 -> full table first) + the replay tests
set -o pipefail
TAG=${1:-rp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for v in 1 0 1; do
  RQ_RP_SMALL=$v timeout -k 10 200 python3 -u scripts/dev/ab_replay.py > "$OUT/ab$v.json" 2>"$OUT/ab$v.err" || { echo "ab $v failed"; tail -5 "$OUT/ab$v.err"; exit 1; }
  echo "small=$v $(cat $OUT/ab$v.json)"
done
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_batch.py tests/test_gpu_replay_chunked.py tests/test_gpu_realdata.py tests/test_gpu_analysis.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
