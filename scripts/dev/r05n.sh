# deferred row stores in the merged sweep: A/B against the stamped build, then the GPU suite
set -o pipefail
export TMPDIR=/tmp
LIBS="librq_base.so librq.so" TAG=r05n bash scripts/dev/ab5.sh > gpurun_out/r05n_ab.txt 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05n_tests.txt 2>&1
