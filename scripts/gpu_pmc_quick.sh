#!/bin/bash
# quick PMC pass for the sweep (two SQ counter groups); usage: scripts/gpu_pmc_quick.sh TAG
set -e -o pipefail
TAG=${1:-q}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
B="bench.py --steps 2 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/p1" -o p1 -- python3 $B > "$OUT/p1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d "$OUT/p2" -o p2 -- python3 $B > "$OUT/p2.log" 2>&1
