set -o pipefail
OUT=gpurun_out/r04fin; mkdir -p $OUT
bash scripts/gpu_pmc.sh r04c5 c5 8192 && \
timeout -k 10 300 python3 -u bench.py --workload c5 > $OUT/c5_bench.log 2>&1 && tail -1 $OUT/c5_bench.log | cut -c1-300 && \
timeout -k 10 300 python3 -u bench.py --workload c4 > $OUT/c4_bench.log 2>&1 && tail -1 $OUT/c4_bench.log | cut -c1-300
