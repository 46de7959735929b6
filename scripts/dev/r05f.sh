set -o pipefail
OUT=gpurun_out/r05f; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 6 --warmup 2 --no-cpu > $OUT/kt.log 2>&1 && tail -1 $OUT/kt.log | cut -c1-200
find $OUT/kt -name "*kernel_trace.csv" | head -3
