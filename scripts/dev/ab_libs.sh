# same-box A/B of several builds on a bench workload: ab_libs.sh WL ROUNDS LIB...
set -o pipefail
WL=$1; N=$2; shift 2
S=$([ "$WL" = c5 ] && echo 2 || echo 20)
for i in $(seq 1 $N); do
  for L in "$@"; do
    RQ_SO_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 bench.py --workload $WL --steps $S --warmup 2 --no-cpu > gpurun_out/abl.log 2>&1 || { echo "$L failed"; tail -3 gpurun_out/abl.log; exit 1; }
    python3 -c "import json; l=json.loads(open('gpurun_out/abl.log').read().strip().splitlines()[-1]); print('$L', round(l['ms_per_step'],3), 'serial', {k: (round(v,3) if isinstance(v, float) else v) for k,v in l['kernels_ms_per_launch_serial'].items() if k != 'launches'})"
  done
done
