set -o pipefail
OUT=gpurun_out/r04q; mkdir -p $OUT
export TMPDIR=/tmp
scripts/gpu_ab_env.sh r04q --workload c5 --steps 3 -- "base=" "colds=RQ_G_COLLDS=1" "b8=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_b8.so" "b6=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_b6.so" "base2="
