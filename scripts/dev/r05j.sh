set -o pipefail
OUT=gpurun_out/r05k; mkdir -p $OUT; export TMPDIR=/tmp
b() { timeout -k 10 300 python3 -u bench.py --no-cpu "$@" > $OUT/b.log 2>&1 && python3 -c "import json; l=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$*', round(l['value']), round(l['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()}, l['sweep_plan']['waves_per_block'], l['sweep_plan']['blocks_per_cu'])"; }
b --steps 20 --warmup 3 && b --steps 20 --warmup 3 --streams 1 && b --workload c5 --steps 4 --warmup 1 && RQ_PIPE=1 b --workload c5 --steps 3 --warmup 1 --replicas 4096 && b --workload c4 --steps 5 --warmup 2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_merge.py tests/test_gpu_configs.py tests/test_gpu_graphs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
