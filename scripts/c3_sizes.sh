#!/bin/bash
# C3 sweep/scan time vs replicas per launch (resident-round effects)
set -o pipefail
for R in ${@:-4096 8192 10000 12288}; do
  timeout -k 10 120 python3 bench.py --replicas $R --steps 5 --warmup 1 --no-cpu > gpurun_out/c3_$R.log 2>&1 || { echo "R=$R failed"; tail -3 gpurun_out/c3_$R.log; exit 1; }
  python3 -c "import json; l=json.loads(open('gpurun_out/c3_$R.log').read().strip().splitlines()[-1]); print($R, round(l['ms_per_step'],3), {k: round(v,3) for k,v in l['kernels_ms_per_launch'].items()}, l['sweep_plan']['waves_per_block'], l['sweep_plan']['blocks_per_cu'])"
done
