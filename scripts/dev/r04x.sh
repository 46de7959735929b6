set -o pipefail
OUT=gpurun_out/r04x; mkdir -p $OUT
export TMPDIR=/tmp
scripts/gpu_ab_env.sh r04x --workload c4 --steps 10 -- "nt=" "plain=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_pl.so" "nt2=" "plain2=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_pl.so"
