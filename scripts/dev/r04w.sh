set -o pipefail
OUT=gpurun_out/r04w; mkdir -p $OUT
export TMPDIR=/tmp
scripts/gpu_ab_env.sh r04w --workload c4 --steps 10 -- "c16k=" "c32k=RQ_PIPE_CHUNK=32000" "c64k=RQ_PIPE_CHUNK=64000" "c128k=RQ_PIPE_CHUNK=128000"
