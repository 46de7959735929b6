# per-kernel stats of the 600-source fast path for two builds (rocprofv3 kernel trace)
set -o pipefail
export TMPDIR=/tmp
for L in librq_base librq; do
  RQ_SO_PATH=$GRAFT_REPO_ROOT/redqueen_amd/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt600_$L -o kt -- python3 scripts/bench_paths.py --only fast_600_sources > gpurun_out/kt600_$L.log 2>&1 || { tail -3 gpurun_out/kt600_$L.log; exit 1; }
  f=$(find gpurun_out/kt600_$L -name "*kernel_stats.csv" | head -1)
  echo "== $L"; cut -d, -f1-4 "$f" | head -8
done
