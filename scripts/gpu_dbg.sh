#!/bin/bash
# Sweep phase breakdown: RQ_SWEEP_DBG=0..4 (1 skip phase C, 2 skip sink updates, 3 skip phase B, 4 skip the fused rank sort)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
for d in 0 1 3 4; do
  RQ_SWEEP_DBG=$d timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu > /tmp/dbg$d.log 2>&1 || { echo "dbg $d failed"; tail -5 /tmp/dbg$d.log; exit 1; }
  python3 -c "import json; l=json.loads(open('/tmp/dbg$d.log').read().strip().splitlines()[-1]); print('dbg', $d, l['kernels_ms_per_launch'], round(l['ms_per_step'],2))"
done
