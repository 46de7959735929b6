# same-box A/B of librq builds on the C5 sweep alone (one stream, 4096 replicas)
set -o pipefail
OUT=gpurun_out/${TAG:-abc5}; mkdir -p $OUT; export TMPDIR=/tmp
b() { L=$1; shift; RQ_SO_PATH=$PWD/redqueen_amd/$L timeout -k 10 300 python3 -u bench.py --no-cpu "$@" > $OUT/b.log 2>&1 && python3 -c "import json; l=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$L $*', round(l['ms_per_step'],3), {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()})"; }
for i in 1 2; do for L in $LIBS; do RQ_PIPE=1 b $L --workload c5 --steps 3 --warmup 1 --replicas 4096 --streams 1 || exit 1; done; done
for L in $LIBS; do b $L --workload c5 --steps 3 --warmup 1 || exit 1; done
