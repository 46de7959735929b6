#!/bin/bash
# Merged-stream general sweep: parity tests, then C5 merged vs windowed (RQ_MRG=0)
# bench lines and the kernel stats of the merged run.  Output: gpurun_out/$TAG.
set -o pipefail
TAG=${1:-mrg}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
TESTS=${TESTS:-"tests/test_gpu_merge.py tests/test_gpu_engine.py tests/test_gpu_configs.py"}
timeout -k 10 500 python3 -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python3 -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > "$OUT/c5_mrg.log" 2>&1 || { echo "c5 mrg failed"; tail -5 "$OUT/c5_mrg.log"; exit 1; }
tail -1 "$OUT/c5_mrg.log"
RQ_MRG=0 timeout -k 10 200 python3 -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > "$OUT/c5_win.log" 2>&1 || { echo "c5 win failed"; tail -5 "$OUT/c5_win.log"; exit 1; }
tail -1 "$OUT/c5_win.log"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5kt" -o kt -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > "$OUT/c5kt.log" 2>&1 || { echo "c5 kt failed"; tail -5 "$OUT/c5kt.log"; exit 1; }
echo "done"
