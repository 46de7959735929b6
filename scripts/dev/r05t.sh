# every GPU ensemble comparison, records into gpurun_out/ens_gpu.jsonl
set -o pipefail
export TMPDIR=/tmp
rm -f gpurun_out/ens_gpu.jsonl
RQ_ENSEMBLE_LOG=$PWD/gpurun_out/ens_gpu.jsonl timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_stats.py tests/test_gpu_significance.py "tests/test_gpu_plugin.py::test_reactive_plugin_beside_redqueen" -q --timeout 600 --timeout-method thread > gpurun_out/ens_gpu.txt 2>&1
