# bitset word loop without segments when the tile has no own event: tests, A/B, serialised sweep
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_configs.py tests/test_gpu_stats.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
LIBS="librq_base.so librq.so" TAG=r05u bash scripts/dev/ab5.sh || exit 1
for WL in c3 c4; do for L in librq_base.so librq.so librq_base.so librq.so; do
  RQ_SO_PATH=$PWD/redqueen_amd/$L AMD_SERIALIZE_KERNEL=3 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$WL -o kts -- python3 bench.py --steps 3 --warmup 1 --no-cpu --workload $WL > $O/${WL}_$L.log 2>&1 || exit 1
  python3 -c "
import csv, glob
for f in glob.glob('$O/k_$WL/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'rq_sweep' in r['Name']: print('$WL $L', r['Name'][:30], round(float(r['AverageNs'])/1e6, 4))"
  rm -rf $O/k_$WL
done; done
