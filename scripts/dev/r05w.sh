# C5 merged sweep compiled for 5 waves per SIMD (RQ_MRG_WPE=5) vs 4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
for i in 1 2; do for L in librq.so librq_w5.so; do
  RQ_SO_PATH=$PWD/redqueen_amd/$L timeout -k 10 400 python3 -u bench.py --no-cpu --workload c5 --steps 3 --warmup 1 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('$L', round(l['ms_per_step'],2), round(l['value']), l['sweep_plan'], {k: round(v,2) for k,v in l['kernels_ms_per_launch'].items()})"
done; done
