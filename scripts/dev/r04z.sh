set -o pipefail
OUT=gpurun_out/r04z; mkdir -p $OUT
export TMPDIR=/tmp
L=$(pwd)/redqueen_amd
scripts/gpu_ab_env.sh r04z --workload c5 --steps 3 -- "base=" "lb768=RQ_SO_PATH=$L/librq_lb768.so" "lb768b8=RQ_SO_PATH=$L/librq_lb768b8.so" "b6=RQ_SO_PATH=$L/librq_b6.so" "base2="
for v in base lb768 lb768b8; do python3 -c "import json; l=json.loads(open('$OUT/bench_$v.log').read().strip().splitlines()[-1]); print('$v', l['sweep_plan'])"; done
