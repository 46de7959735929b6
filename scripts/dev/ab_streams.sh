# bench.py caller streams (one chunk per call) A/B on C3
set -o pipefail
for i in 1 2; do for S in 2 3 4; do
timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu --streams $S > gpurun_out/abs.log 2>&1 || { tail -3 gpurun_out/abs.log; exit 1; }
python3 -c "import json; l=json.loads(open('gpurun_out/abs.log').read().strip().splitlines()[-1]); print('streams $S', round(l['value']), round(l['ms_per_step'],3), l['roofline']['frac'])"
done; done
