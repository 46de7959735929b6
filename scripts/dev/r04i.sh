set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
export TMPDIR=/tmp
summ() {
  python3 - $1 <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "merge" in k or "gen" in k:
        m = {c: sum(v) / len(v) for c, v in d.items()}
        rb = 128 * m.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0)
        print(sys.argv[1].split("/")[-1], k[:30], "read %.4g" % rb, "write %.4g" % (m.get("WRITE_SIZE", 0) * 1024))
PY
}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_merge.py tests/test_gpu_engine.py tests/test_gpu_stats.py -x -q -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
for v in base g8 nont; do
  case $v in base) unset RQ_SO_PATH;; g8) export RQ_SO_PATH=$PWD/redqueen_amd/librq_g8.so;; nont) export RQ_SO_PATH=$PWD/redqueen_amd/librq_nont.so;; esac
  B="bench.py --steps 2 --warmup 1 --no-cpu --workload c3"
  timeout -k 10 -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/${v}_r -o x -- python3 $B > $OUT/${v}_r.log 2>&1 || { echo $v failed; tail -5 $OUT/${v}_r.log; exit 1; }
  summ $OUT/${v}_r
  timeout -k 10 -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${v}_w -o x -- python3 $B > $OUT/${v}_w.log 2>&1 || { echo w failed; exit 1; }
  summ $OUT/${v}_w
done
unset RQ_SO_PATH
scripts/gpu_ab_env.sh r04i -- "base=" "g8=RQ_SO_PATH=$PWD/redqueen_amd/librq_g8.so" "nont=RQ_SO_PATH=$PWD/redqueen_amd/librq_nont.so" && \
scripts/gpu_ab_env.sh r04i --workload c5 --steps 4 -- "c5base=" "c5g8=RQ_SO_PATH=$PWD/redqueen_amd/librq_g8.so"
