#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) + a kernel-trace pass for ONE
# bench_paths.py section, so each secondary workload gets its own summary.
# usage: scripts/gpu_paths_pmc.sh TAG SECTION   -> gpurun_out/pmcp_TAG_SECTION/summary.json
set -o pipefail
TAG=${1:-run}
SEC=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmcp_${TAG}_$SEC
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
B="scripts/bench_paths.py --reps 2 --only $SEC"
P="--output-format csv"
run() {   # name, counters...
  local n=$1; shift
  if [ "$n" = kt ]; then
    timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats $P -d "$OUT/$n" -o $n -- python3 $B > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -5 "$OUT/$n.log"; return 1; }
  else
    timeout -k 10 -s KILL 200 rocprofv3 --pmc "$@" $P -d "$OUT/$n" -o $n -- python3 $B > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -5 "$OUT/$n.log"; return 1; }
  fi
}
run kt && run p3 FETCH_SIZE && run p4 WRITE_SIZE && \
run p5 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum && \
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU && \
run p2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
python3 scripts/pmc_summary.py "$OUT" workload=$SEC "command=scripts/gpu_paths_pmc.sh $TAG $SEC ($B)" > "$OUT/summary.txt" && grep -E "^rq_|^_meta" "$OUT/summary.txt" | cut -c1-300
