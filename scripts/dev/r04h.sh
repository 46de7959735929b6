set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
export TMPDIR=/tmp
summ() {
  python3 - $1 <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "merge" in k or "gen" in k or "sweep" in k:
        m = {c: sum(v) / len(v) for c, v in d.items()}
        rb = 128 * m.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0)
        print(sys.argv[1].split("/")[-1], k[:30], "read bytes by req %.4g" % rb, "write %.4g" % (m.get("WRITE_SIZE", 0) * 1024))
PY
}
for v in ntl nt; do
  if [ $v = nt ]; then export RQ_SO_PATH=$PWD/redqueen_amd/librq_nt.so; fi
  for wl in c3 c5; do
    B="bench.py --steps 2 --warmup 1 --no-cpu --workload $wl"
    timeout -k 10 -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/${v}_$wl -o x -- python3 $B > $OUT/${v}_$wl.log 2>&1 || { echo $v $wl failed; tail -5 $OUT/${v}_$wl.log; exit 1; }
    summ $OUT/${v}_$wl
  done
  timeout -k 10 -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${v}_c3w -o x -- python3 bench.py --steps 2 --warmup 1 --no-cpu --workload c3 > $OUT/${v}_c3w.log 2>&1 || { echo w failed; exit 1; }
  summ $OUT/${v}_c3w
done
unset RQ_SO_PATH
scripts/gpu_ab_env.sh r04h -- "ntl=" "nt=RQ_SO_PATH=$PWD/redqueen_amd/librq_nt.so" && \
scripts/gpu_ab_env.sh r04h --workload c5 --steps 4 -- "c5ntl=" "c5nt=RQ_SO_PATH=$PWD/redqueen_amd/librq_nt.so"
