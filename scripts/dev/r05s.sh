# C3 bench: caller streams 1 / 2 / 3 / 4, three rounds each, same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
for i in 1 2 3; do for S in 2 3 4; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --steps 30 --warmup 3 --streams $S > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('streams $S', round(l['ms_per_step'],3), round(l['value']/1e6,3))"
done; done
