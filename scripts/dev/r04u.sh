set -o pipefail
OUT=gpurun_out/r04u; mkdir -p $OUT
export TMPDIR=/tmp
scripts/gpu_ab_env.sh r04u --workload c4 --steps 10 -- "base=" "fwm0=RQ_FWM=0" "mrg0=RQ_MRG=0" "pipe1=RQ_PIPE=1"
for v in base fwm0 mrg0 pipe1; do python3 -c "import json; l=json.loads(open('$OUT/bench_$v.log').read().strip().splitlines()[-1]); print('$v', l.get('launches_per_step'), l['sweep_plan'])"; done
