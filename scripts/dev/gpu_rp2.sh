#!/bin/bash
# replay small-table tier on a 1024-df batch (4 workgroups per CU)
set -o pipefail
TAG=${1:-rp2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for v in 1 0 1 0; do
  RQ_AB_NDF=1024 RQ_RP_SMALL=$v timeout -k 10 200 python3 -u scripts/dev/ab_replay.py > "$OUT/ab$v.json" 2>"$OUT/ab$v.err" || { echo "ab $v failed"; tail -5 "$OUT/ab$v.err"; exit 1; }
  echo "small=$v $(cat $OUT/ab$v.json)"
done
