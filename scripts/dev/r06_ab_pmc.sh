#!/bin/bash
# A/B of two librq builds: per-phase clock split (diagnostic builds) and one SQ counter
# pass per build on the C3 bench (kernel-level VALU / SALU / LDS instruction counts).
# usage: scripts/dev/r06_ab_pmc.sh TAG LIB_A LIB_B CLK_A CLK_B
set -o pipefail
TAG=$1; A=$2; B=$3; CA=$4; CB=$5
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for L in $CA $CB; do
  RQ_SO_PATH=$ROOT/$L timeout -k 10 120 python3 scripts/phase_clock.py > "$OUT/clk_$(basename $L).log" 2>&1 || { echo "clk $L failed"; tail -3 "$OUT/clk_$(basename $L).log"; exit 1; }
  echo "$L"; tail -2 "$OUT/clk_$(basename $L).log"
done
for L in $A $B; do
  N=$(basename $L .so)
  RQ_SO_PATH=$ROOT/$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d "$OUT/pmc_$N" -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu --streams 1 > "$OUT/pmc_$N.log" 2>&1 || { echo "pmc $L failed"; tail -3 "$OUT/pmc_$N.log"; exit 1; }
  python3 - "$OUT/pmc_$N" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    if "rq_sweep" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / n[(k, c)] / 1e6, 2) for c, v in d.items()})
PY
done
