#!/bin/bash
# Profile the bench workload on the GPU box: kernel trace + PMC passes.
# usage: scripts/gpu_profile.sh TAG   (outputs under gpurun_out/prof_TAG/)
set -e -o pipefail
TAG=${1:-run}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
B="bench.py --steps 3 --warmup 1 --no-cpu"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 $B > "$OUT/kt.log" 2>&1
echo "kt done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/p1" -o p1 -- python3 $B > "$OUT/p1.log" 2>&1
echo "p1 done"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d "$OUT/p2" -o p2 -- python3 $B > "$OUT/p2.log" 2>&1
echo "p2 done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/p3" -o p3 -- python3 $B > "$OUT/p3.log" 2>&1
echo "p3 done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/p4" -o p4 -- python3 $B > "$OUT/p4.log" 2>&1
echo "p4 done"
