set -o pipefail
OUT=gpurun_out/r05g; mkdir -p $OUT; export TMPDIR=/tmp
b() { timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu "$@" > $OUT/b.log 2>&1 && python3 -c "import json; l=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$*', round(l['value']), round(l['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()})"; }
b --streams 1 && b && b --streams 3 && b --dist && b --streams 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 6 --warmup 2 --no-cpu > $OUT/kt.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_engine.py tests/test_gpu_merge.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
