set -o pipefail
OUT=gpurun_out/r04v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error" $OUT/pytest1.log | tail -30; [ $rc = 0 ] || { tail -40 $OUT/pytest1.log; exit 1; }
scripts/gpu_ab_env.sh r04v --workload c4 --steps 10 -- "small=" "bucket=RQ_MERGE_SMALL=0"
scripts/gpu_ab_env.sh r04v --workload c3 --steps 20 -- "c3="
