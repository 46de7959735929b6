set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
export TMPDIR=/tmp
for R in 8192 12288 16384; do
  timeout -k 10 300 python3 -u bench.py --workload c5 --replicas $R --steps 3 --warmup 1 --no-cpu > $OUT/c5_$R.log 2>&1 || { tail -5 $OUT/c5_$R.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$OUT/c5_$R.log').read().strip().splitlines()[-1]); print($R, round(l['value']), round(l['ms_per_step'],1), l['kernels_ms_per_launch'], l['sweep_plan']['chunk'], l.get('launches_per_step'))"
done
RQ_PIPE=1 timeout -k 10 300 python3 -u bench.py --workload c5 --replicas 4096 --steps 3 --warmup 1 --no-cpu > $OUT/c5_pipe1.log 2>&1 || { tail -5 $OUT/c5_pipe1.log; exit 1; }
python3 -c "import json; l=json.loads(open('$OUT/c5_pipe1.log').read().strip().splitlines()[-1]); print('pipe1 4096', round(l['value']), round(l['ms_per_step'],1), l['kernels_ms_per_launch'], l['sweep_plan']['chunk'])"
