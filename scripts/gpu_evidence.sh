#!/bin/bash
# Round evidence for the bench workloads in one GPU call: per workload the stamped PMC
# summary (scripts/gpu_pmc.sh: kernel trace, serialised trace, counter passes), copied
# into profiles/ on the box first so the bench lines report its traffic, then the bench
# line and its rocprofv3 kernel stats.  Outputs land in gpurun_out/TAG; copy them into
# profiles/ (RND prefix).  usage: RND=r05 scripts/gpu_evidence.sh TAG [workloads]
set -o pipefail
TAG=${1:-ev}
WLS=${2:-"c3 c5 c4"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
RND=${RND:-r06}
for WL in $WLS; do
  R=$([ "$WL" = c5 ] && echo 8192 || ([ "$WL" = c4 ] && echo 1000 || echo 10000))
  S=$([ "$WL" = c5 ] && echo 3 || echo 20)
  scripts/gpu_pmc.sh ${TAG}_pmc_$WL $WL $R > "$OUT/pmc_$WL.log" 2>&1 || { echo "pmc $WL failed"; tail -5 "$OUT/pmc_$WL.log"; exit 1; }
  cp "$ROOT/gpurun_out/pmc_${TAG}_pmc_$WL/summary.json" "profiles/${RND}_${WL}_pmc_summary.json"
  cp "$ROOT/gpurun_out/pmc_${TAG}_pmc_$WL/summary.txt" "$OUT/${WL}_pmc_summary.txt"
  # the serialised kernel trace's stats (AMD_SERIALIZE_KERNEL=3: every launch alone on the
  # chip, the duration bench.py's serial probe and roofline use)
  find "$ROOT/gpurun_out/pmc_${TAG}_pmc_$WL/kts" -name "*kernel_stats.csv" -exec cp {} "$OUT/${WL}_kernel_stats_serial.csv" \;
  echo "pmc $WL ok"
  CPU=$([ "$WL" = c3 ] && echo "" || echo "--no-cpu")
  timeout -k 10 400 python3 -u bench.py --workload $WL --steps $S --warmup 2 $CPU > "$OUT/${WL}_bench.log" 2>&1 || { echo "$WL bench failed"; tail -5 "$OUT/${WL}_bench.log"; exit 1; }
  tail -1 "$OUT/${WL}_bench.log" > "$OUT/${WL}_bench.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${WL}kt" -o kt -- python3 bench.py --workload $WL --steps $S --warmup 2 --no-cpu > "$OUT/${WL}kt.log" 2>&1 || { echo "$WL kt failed"; tail -5 "$OUT/${WL}kt.log"; exit 1; }
  echo "$WL bench + kt ok"
done
if [ -z "${2:-}" ]; then
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 2 --no-cpu --dist > "$OUT/c3_bench_dist.log" 2>&1 || { echo "dist bench failed"; tail -5 "$OUT/c3_bench_dist.log"; exit 1; }
  tail -1 "$OUT/c3_bench_dist.log" > "$OUT/c3_bench_dist.json"
  echo "dist bench ok"
fi
