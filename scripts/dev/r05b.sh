set -o pipefail
OUT=gpurun_out/r05b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dist.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu --dist > $OUT/bench_dist.log 2>&1 && tail -1 $OUT/bench_dist.log | cut -c1-300
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench2.log 2>&1 && tail -1 $OUT/bench2.log | cut -c1-300
