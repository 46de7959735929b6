set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_dist.py tests/test_gpu_inference.py tests/test_gpu_significance.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04d/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r04d/pytest.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04d -- "c3=" "c3nt=RQ_SO_PATH=$PWD/redqueen_amd/librq_nt.so" "c2k=RQ_PIPE_CHUNK=2000" "c2500=RQ_PIPE_CHUNK=2500" "c3334=RQ_PIPE_CHUNK=3334" "p3c2k=RQ_PIPE=3 RQ_PIPE_CHUNK=2000" "p1=RQ_PIPE=1" && \
timeout -k 10 600 python3 -u scripts/bench_inference.py --out gpurun_out/r04d/inference.json > gpurun_out/r04d/inference.log 2>&1 && tail -8 gpurun_out/r04d/inference.log
