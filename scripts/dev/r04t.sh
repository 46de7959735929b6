set -o pipefail
OUT=gpurun_out/r04t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_graphs.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" $OUT/pytest1.log | tail -20; [ $rc = 0 ] || { tail -40 $OUT/pytest1.log; exit 1; }
