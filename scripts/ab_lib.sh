#!/bin/bash
# same-box A/B of two builds on a bench workload: ab_lib.sh LIB_A LIB_B [rounds] [workload]
# prints ms/step, the live per-launch kernel times and the serialised probe's sweep time
set -o pipefail
A=$1; B=$2; N=${3:-3}; WL=${4:-c3}
S=$([ "$WL" = c5 ] && echo 2 || echo 10)
for i in $(seq 1 $N); do
  for L in $A $B; do
    RQ_SO_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 bench.py --workload $WL --steps $S --warmup 2 --no-cpu > gpurun_out/ab.log 2>&1 || { echo "$L failed"; tail -3 gpurun_out/ab.log; exit 1; }
    python3 -c "import json; l=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$L', round(l['ms_per_step'],3), {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()}, 'serial', {k: (round(v,3) if isinstance(v, float) else v) for k,v in l['kernels_ms_per_launch_serial'].items()})"
  done
done
