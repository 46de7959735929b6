set -o pipefail
OUT=gpurun_out/r05l; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
b() { timeout -k 10 300 python3 -u bench.py --no-cpu "$@" > $OUT/b.log 2>&1 && python3 -c "import json; l=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$*', round(l['value']), round(l['ms_per_step'],3), {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()})"; }
b --steps 20 --warmup 3 && b --workload c5 --steps 4 --warmup 1 && b --workload c4 --steps 5 --warmup 2
