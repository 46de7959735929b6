set -o pipefail
OUT=gpurun_out/r05d; mkdir -p $OUT; export TMPDIR=/tmp
b() { timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu "$@" > $OUT/b.log 2>&1 && python3 -c "import json; l=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$*', round(l['ms_per_step'],3), 'ms/step', {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()})"; }
b && b --dist && RQ_NOGATHER=1 b --dist && GPU_MAX_HW_QUEUES=8 b --dist && GPU_MAX_HW_QUEUES=8 b
