set -o pipefail
OUT=gpurun_out/r05e; mkdir -p $OUT; export TMPDIR=/tmp
RQ_ENSEMBLE_LOG=$PWD/$OUT/ens.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-250
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu --dist > $OUT/bench_dist.log 2>&1 && tail -1 $OUT/bench_dist.log | cut -c1-250
