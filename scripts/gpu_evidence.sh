#!/bin/bash
# Round evidence in one GPU call: PMC summaries first (copied into profiles/ on the
# box so the bench lines report their traffic), then the GPU suite, the C3 and C5
# bench lines with their rocprofv3 kernel stats, and the secondary paths (replay,
# scan, log expand).  Everything lands in gpurun_out/TAG; copy it into profiles/.
# usage: scripts/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
RND=${RND:-r02}
scripts/gpu_pmc.sh ${TAG}_pmc_c3 c3 10000 > "$OUT/pmc_c3.log" 2>&1 || { echo "pmc c3 failed"; tail -5 "$OUT/pmc_c3.log"; exit 1; }
cp "$ROOT/gpurun_out/pmc_${TAG}_pmc_c3/summary.json" "profiles/${RND}_c3_pmc_summary.json"
echo "pmc c3 ok"
scripts/gpu_pmc.sh ${TAG}_pmc_c5 c5 4096 > "$OUT/pmc_c5.log" 2>&1 || { echo "pmc c5 failed"; tail -5 "$OUT/pmc_c5.log"; exit 1; }
cp "$ROOT/gpurun_out/pmc_${TAG}_pmc_c5/summary.json" "profiles/${RND}_c5_pmc_summary.json"
echo "pmc c5 ok"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -u bench.py > "$OUT/c3_bench.log" 2>&1 || { echo "c3 bench failed"; tail -5 "$OUT/c3_bench.log"; exit 1; }
tail -1 "$OUT/c3_bench.log" > "$OUT/c3_bench.json"
echo "c3 bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3kt" -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/c3kt.log" 2>&1 || { echo "c3 kt failed"; tail -5 "$OUT/c3kt.log"; exit 1; }
echo "c3 kt ok"
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 3 --warmup 1 > "$OUT/c5_bench.log" 2>&1 || { echo "c5 bench failed"; tail -5 "$OUT/c5_bench.log"; exit 1; }
tail -1 "$OUT/c5_bench.log" > "$OUT/c5_bench.json"
echo "c5 bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5kt" -o kt -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > "$OUT/c5kt.log" 2>&1 || { echo "c5 kt failed"; tail -5 "$OUT/c5kt.log"; exit 1; }
echo "c5 kt ok"
timeout -k 10 300 python3 scripts/bench_paths.py --reps 5 > "$OUT/paths.json" 2> "$OUT/paths.err" || { echo "paths failed"; tail -5 "$OUT/paths.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pathskt" -o kt -- python3 scripts/bench_paths.py --reps 3 > "$OUT/pathskt.log" 2>&1 || { echo "paths kt failed"; tail -5 "$OUT/pathskt.log"; exit 1; }
echo "paths ok"
# HBM bytes of the secondary paths' kernels (replay, scan, log expand): FETCH / WRITE passes
P="--output-format csv"
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE $P -d "$OUT/pathsp3" -o p3 -- python3 scripts/bench_paths.py --reps 1 > "$OUT/pathsp3.log" 2>&1 || { echo "paths fetch failed"; tail -5 "$OUT/pathsp3.log"; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE $P -d "$OUT/pathsp4" -o p4 -- python3 scripts/bench_paths.py --reps 1 > "$OUT/pathsp4.log" 2>&1 || { echo "paths write failed"; tail -5 "$OUT/pathsp4.log"; exit 1; }
mkdir -p "$OUT/pathspmc" && mv "$OUT/pathsp3" "$OUT/pathsp4" "$OUT/pathspmc/"
python3 scripts/pmc_summary.py "$OUT/pathspmc" workload=paths "command=scripts/bench_paths.py --reps 1" > "$OUT/paths_pmc_summary.txt" || { echo "paths pmc summary failed"; exit 1; }
cp "$OUT/pathspmc/summary.json" "$OUT/paths_pmc_summary.json"
echo "paths pmc ok"
