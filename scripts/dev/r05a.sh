set -o pipefail
OUT=gpurun_out/r05a; mkdir -p $OUT; export TMPDIR=/tmp
RQ_ENSEMBLE_LOG=$PWD/$OUT/ens.jsonl timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stats.py tests/test_gpu_dist.py "tests/test_gpu_significance.py::test_ensemble_vs_reference" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu --dist > $OUT/bench_dist.log 2>&1 && tail -1 $OUT/bench_dist.log | cut -c1-400
