set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_merge.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; tail -3 $OUT/pytest1.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04p --workload c5 --steps 3 -- "orig=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_orig.so" "sk0=RQ_SKIP=0" "sk1=" "sk1b="
scripts/gpu_ab_env.sh r04p --workload c3 -- "c3orig=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_orig.so" "c3="
