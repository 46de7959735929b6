set -o pipefail
OUT=gpurun_out/r05paths; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/bench_paths.py --reps 5 > $OUT/paths.json 2> $OUT/paths.err || { echo "paths failed"; tail -5 $OUT/paths.err; exit 1; }
echo paths ok
for SEC in replay_batch replay_batch_1024; do scripts/gpu_paths_pmc.sh r05 $SEC > $OUT/pmc_$SEC.log 2>&1 || { echo "pmc $SEC failed"; tail -5 $OUT/pmc_$SEC.log; exit 1; }; echo "pmc $SEC ok"; done
