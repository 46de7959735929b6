#!/bin/bash
# Sweep phase breakdown (RQ_SWEEP_DBG) + PMC passes on the bench workload.  usage: scripts/gpu_breakdown.sh TAG
set -o pipefail
TAG=${1:-bd}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
B="bench.py --steps 3 --warmup 1 --no-cpu"
for d in 0 1 2 3; do
  RQ_SWEEP_DBG=$d timeout -k 10 200 python3 $B > "$OUT/dbg$d.log" 2>&1 || { echo "dbg $d failed"; tail -5 "$OUT/dbg$d.log"; exit 1; }
  python3 -c "import json,sys; l=json.loads(open('$OUT/dbg$d.log').read().strip().splitlines()[-1]); print('dbg', $d, l['kernels_ms_per_launch'], l['ms_per_step'])"
done
P="--output-format csv"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU $P -d "$OUT/p1" -o p1 -- python3 $B > "$OUT/p1.log" 2>&1 || { echo p1 failed; tail -5 "$OUT/p1.log"; exit 1; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM $P -d "$OUT/p2" -o p2 -- python3 $B > "$OUT/p2.log" 2>&1 || { echo p2 failed; tail -5 "$OUT/p2.log"; exit 1; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE $P -d "$OUT/p3" -o p3 -- python3 $B > "$OUT/p3.log" 2>&1 || { echo p3 failed; tail -5 "$OUT/p3.log"; exit 1; }
timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE $P -d "$OUT/p4" -o p4 -- python3 $B > "$OUT/p4.log" 2>&1 || { echo p4 failed; tail -5 "$OUT/p4.log"; exit 1; }
python3 scripts/pmc_summary.py "$OUT"
