set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_configs.py tests/test_gpu_graphs.py tests/test_gpu_stats.py -x -q -k "not c4_corners" --timeout 300 --timeout-method thread > gpurun_out/r04f/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r04f/pytest.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04f --workload c5 --steps 5 -- "c5=" || exit 1
bash scripts/dev/r04e.sh
