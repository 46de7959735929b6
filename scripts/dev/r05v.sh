# C5 step: pipelined chunk size (4096 default, 2048, 1366)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
for i in 1 2; do for C in 0 2048 1366; do
  if [ $C = 0 ]; then unset RQ_PIPE_CHUNK; else export RQ_PIPE_CHUNK=$C; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu --workload c5 --steps 3 --warmup 1 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('chunk $C', round(l['ms_per_step'],2), round(l['value']), {k: round(v,2) for k,v in l['kernels_ms_per_launch'].items()})"
done; done
