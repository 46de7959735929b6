set -o pipefail
scripts/gpu_calib_half.sh r04_calib2 && \
scripts/gpu_ab_env.sh r04c --workload c5 --steps 5 -- "c5=" "c5p1=RQ_PIPE=1" "c5o0=RQ_ORDER=0" && \
scripts/gpu_ab_env.sh r04c --workload c4 --steps 5 -- "c4=" "c4p1=RQ_PIPE=1" && \
timeout -k 10 600 python3 -u scripts/bench_inference.py --out gpurun_out/r04c/inference.json > gpurun_out/r04c/inference.log 2>&1 && tail -8 gpurun_out/r04c/inference.log && \
scripts/gpu_pmc.sh r04_c3 c3 10000
