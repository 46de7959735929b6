set -o pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04k --workload c5 --steps 4 -- "c5=" && scripts/gpu_ab_env.sh r04k -- "c3="
