# sweep VALU / SALU / LDS instruction counts with phase C (dbg 1) or the controller (dbg 3) skipped
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
B="bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu --workload ${WL:-c3} ${EXTRA:-}"
for D in 0 1 3; do
  RQ_SWEEP_DBG=$D timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $O/d$D -o p -- python3 $B > $O/d$D.log 2>&1 || { tail -5 $O/d$D.log; exit 1; }
  python3 - $O/d$D $D <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if "rq_sweep" in r["Kernel_Name"]:
            acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
k = n['SQ_WAVES'] or 1
print('dbg', sys.argv[2], {c: round(v / n[c]) for c, v in sorted(acc.items())})
PY
done
