set -o pipefail
OUT=gpurun_out/r04fin; mkdir -p $OUT
bash scripts/gpu_round.sh r04fin && bash scripts/gpu_pmc.sh r04c3 c3 10000 && bash scripts/gpu_pmc.sh r04c5 c5 8192 && bash scripts/gpu_pmc.sh r04c4 c4 1000 && \
timeout -k 10 300 python3 -u bench.py --workload c5 > $OUT/c5_bench.log 2>&1 && tail -1 $OUT/c5_bench.log | cut -c1-200 && \
timeout -k 10 300 python3 -u bench.py --workload c4 > $OUT/c4_bench.log 2>&1 && tail -1 $OUT/c4_bench.log | cut -c1-200
