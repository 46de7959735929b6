#!/bin/bash
# phase clocks: the merged fused sweep on C3, the merge on C3 and C5
set -o pipefail
TAG=${1:-clk}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export RQ_SO_PATH=$ROOT/redqueen_amd/librq_mclk.so
timeout -k 10 200 python3 -u scripts/phase_clock.py > "$OUT/sweep.log" 2>&1 || { echo "sweep clock failed"; tail -5 "$OUT/sweep.log"; exit 1; }
grep -v amdgpu.ids "$OUT/sweep.log"
RQ_WL=c3 timeout -k 10 200 python3 -u scripts/dev/merge_clock.py > "$OUT/m3.log" 2>&1 || { echo "m3 failed"; tail -5 "$OUT/m3.log"; exit 1; }
grep -v amdgpu.ids "$OUT/m3.log"
RQ_WL=c5 timeout -k 10 200 python3 -u scripts/dev/merge_clock.py > "$OUT/m5.log" 2>&1 || { echo "m5 failed"; tail -5 "$OUT/m5.log"; exit 1; }
grep -v amdgpu.ids "$OUT/m5.log"
