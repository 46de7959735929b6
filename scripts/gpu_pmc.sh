#!/bin/bash
# PMC passes on the bench workload (one counter group per rocprofv3 run, as the
# gfx950 slot limits require) + a kernel-trace pass; summary -> gpurun_out/pmc_TAG/summary.json
# usage: scripts/gpu_pmc.sh TAG [WORKLOAD [REPLICAS]]   (defaults c3 10000)
set -o pipefail
TAG=${1:-run}
WL=${2:-c3}
R=${3:-$([ "$WL" = c5 ] && echo 4096 || echo 10000)}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
B="bench.py --steps 3 --warmup 1 --no-cpu --workload $WL --replicas $R"
# the sweep variant the plan picks (recorded with the counters; bench.py matches on it)
V=$(timeout -k 10 120 python3 -c "
import bench
from redqueen_amd import engine
so, _ = bench.workload('$WL')
g = engine.Graph(so['src_id'], so['other_sources'], so['sink_ids'], so['edge_list'], so['end_time'])
print(g.run('opt', q=so['q'], s=so['s'], n_rep=$R, randomize=True, plan_only=True)['variant'])") || { echo plan failed; exit 1; }
P="--output-format csv"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats $P -d "$OUT/kt" -o kt -- python3 $B > "$OUT/kt.log" 2>&1 || { echo kt failed; tail -5 "$OUT/kt.log"; exit 1; }
echo "kt ok"
# every kernel alone on the chip (the serialised durations of pmc_summary.py's serial_avg_ns)
AMD_SERIALIZE_KERNEL=3 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats $P -d "$OUT/kts" -o kts -- python3 $B > "$OUT/kts.log" 2>&1 || { echo kts failed; tail -5 "$OUT/kts.log"; exit 1; }
echo "kts ok"
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE $P -d "$OUT/p3" -o p3 -- python3 $B > "$OUT/p3.log" 2>&1 || { echo p3 failed; tail -5 "$OUT/p3.log"; exit 1; }
echo "fetch ok"
timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE $P -d "$OUT/p4" -o p4 -- python3 $B > "$OUT/p4.log" 2>&1 || { echo p4 failed; tail -5 "$OUT/p4.log"; exit 1; }
echo "write ok"
# read requests by size: exact read bytes for any access width (FETCH_SIZE tallies every
# request as 64 B: x2 is exact only for whole-line reads, profiles/r04_calib_half.txt)
timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum $P -d "$OUT/p5" -o p5 -- python3 $B > "$OUT/p5.log" 2>&1 || { echo p5 failed; tail -5 "$OUT/p5.log"; exit 1; }
echo "rdreq ok"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU $P -d "$OUT/p1" -o p1 -- python3 $B > "$OUT/p1.log" 2>&1 || { echo p1 failed; tail -5 "$OUT/p1.log"; exit 1; }
echo "sq1 ok"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT $P -d "$OUT/p2" -o p2 -- python3 $B > "$OUT/p2.log" 2>&1 || { echo p2 failed; tail -5 "$OUT/p2.log"; exit 1; }
echo "sq2 ok"
python3 scripts/pmc_summary.py "$OUT" workload=$WL replicas=$R variant=$V "command=scripts/gpu_pmc.sh $TAG ($B)" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
