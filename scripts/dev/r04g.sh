set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 1 --no-cpu --workload c3"
for v in base nt; do
  if [ $v = nt ]; then export RQ_SO_PATH=$PWD/redqueen_amd/librq_nt.so; fi
  timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/$v -o $v -- python3 $B > $OUT/$v.log 2>&1 || { echo $v failed; tail -5 $OUT/$v.log; exit 1; }
  python3 - $OUT/$v <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "merge" in k or "gen" in k or "sweep" in k:
        m = {c: sum(v) / len(v) for c, v in d.items()}
        print(sys.argv[1].split("/")[-1], k[:30], "read bytes by req %.4g" % (128 * m.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0)))
PY
done
