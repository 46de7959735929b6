set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 60 rocprofv3 -L > gpurun_out/r04b/counters.txt 2>&1 || rocprofv3 --list-avail > gpurun_out/r04b/counters.txt 2>&1 || true
grep -i "TCC_EA0_RD\|TCC_EA_RD\|TCC_BUBBLE\|TCC_EA0_WR" gpurun_out/r04b/counters.txt | head -30
scripts/gpu_ab_env.sh r04b -- "c3=" "c3w5=RQ_SO_PATH=$PWD/redqueen_amd/librq_fwm5.so" "c3p1=RQ_PIPE=1" && \
scripts/gpu_ab_env.sh r04b --workload c5 --steps 5 -- "c5=" "c5p1=RQ_PIPE=1" "c5p1o0=RQ_PIPE=1 RQ_ORDER=0" "c5o0=RQ_ORDER=0" && \
scripts/gpu_ab_env.sh r04b --workload c4 --steps 5 -- "c4=" "c4p1=RQ_PIPE=1" && \
timeout -k 10 600 python3 -u scripts/bench_inference.py --out gpurun_out/r04b/inference.json > gpurun_out/r04b/inference.log 2>&1; tail -8 gpurun_out/r04b/inference.log
