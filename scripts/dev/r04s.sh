set -o pipefail
OUT=gpurun_out/r04s; mkdir -p $OUT
export TMPDIR=/tmp
scripts/gpu_ab_env.sh r04s --workload c3 --steps 30 -- "nt1=" "nt0=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_nt0.so" "nt1b=" "nt0b=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_nt0.so"
scripts/gpu_ab_env.sh r04s --workload c5 --steps 3 -- "c5nt1=" "c5nt0=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_nt0.so"
