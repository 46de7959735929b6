# same-box A/B of librq builds on the 256-df replay batch (scripts/bench_paths.py)
set -o pipefail
OUT=gpurun_out/${TAG:-abrp}; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2; do for L in $LIBS; do
  RQ_SO_PATH=$PWD/redqueen_amd/$L timeout -k 10 300 python3 -u scripts/bench_paths.py --reps 5 --only ${SEC:-replay_batch} > $OUT/p.json 2> $OUT/p.err || { tail -5 $OUT/p.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$OUT/p.json'))
for k,v in d.items():
    if isinstance(v, dict) and 'ms' in str(v): print('$L', k, {a: (round(b,4) if isinstance(b,float) else b) for a,b in v.items() if not isinstance(b,(list,dict))})
"
done; done
