set -o pipefail
OUT=gpurun_out/r04y; mkdir -p $OUT
export TMPDIR=/tmp
RQ_SO_PATH=$(pwd)/redqueen_amd/librq_ept.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; tail -2 $OUT/pytest1.log; [ $rc = 0 ] || { tail -40 $OUT/pytest1.log; exit 1; }
scripts/gpu_ab_env.sh r04y --workload c4 --steps 10 -- "base=" "ept8=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_ept.so" "ept4=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_ept4.so" "base2="
