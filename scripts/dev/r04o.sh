set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_merge.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; tail -3 $OUT/pytest1.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04o --workload c5 --steps 3 -- "sk1=" "sk0=RQ_SKIP=0" "sk1b="
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
