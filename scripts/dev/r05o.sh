# serialised kernel durations, stamped build vs deferred row stores (C3, C4), + the phase clock
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
for WL in c3 c4; do for L in librq_base.so librq.so librq_base.so librq.so; do
  RQ_SO_PATH=$PWD/redqueen_amd/$L AMD_SERIALIZE_KERNEL=3 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$WL -o kts -- python3 bench.py --steps 3 --warmup 1 --no-cpu --workload $WL > $O/${WL}_$L.log 2>&1 || exit 1
  echo "== $WL $L"; python3 -c "
import csv, glob
for f in glob.glob('$O/k_$WL/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'rq_' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 4), round(float(r['MinNs'])/1e6, 4))"
  rm -rf $O/k_$WL
done; done
