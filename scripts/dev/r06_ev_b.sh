#!/bin/bash
# round-6 evidence, part B: the stamped C5 evidence, the secondary paths and the PMC
# summaries of the event-log sweep and the 256-df replay
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ev06b
mkdir -p "$OUT"
cd "$ROOT"
RND=r06 bash scripts/gpu_evidence.sh ev06b "c5" || exit 1
timeout -k 10 400 python3 -u scripts/bench_paths.py > "$OUT/paths.json" 2> "$OUT/paths.err" || { echo "paths failed"; tail -5 "$OUT/paths.err"; exit 1; }
echo "paths ok"
for SEC in sweep_event_log replay_batch; do
  bash scripts/gpu_paths_pmc.sh ev06 $SEC > "$OUT/pmcp_$SEC.log" 2>&1 || { echo "pmc $SEC failed"; tail -5 "$OUT/pmcp_$SEC.log"; exit 1; }
  echo "pmc $SEC ok"
done
