set -o pipefail
OUT=gpurun_out/r05m; mkdir -p $OUT; export TMPDIR=/tmp
b() { timeout -k 10 300 python3 -u bench.py --no-cpu "$@" > $OUT/b.log 2>&1 && python3 -c "import json; l=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$*', round(l['value']), round(l['ms_per_step'],3), l['launches_per_step'], {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()})"; }
for i in 1 2; do b --workload c5 --steps 4 --warmup 2 --streams 1 && b --workload c5 --steps 4 --warmup 2 --streams 2 || exit 1; done
