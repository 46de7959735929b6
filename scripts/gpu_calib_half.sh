#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of half-line (64-B per lane) reads and writes
# (scripts/micro/fetch_half) on the GPU box.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-calib_half}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d "$OUT/RDREQ" -o RDREQ -- scripts/micro/fetch_half > "$OUT/RDREQ.log" 2>&1 || { echo calib RDREQ failed; tail -5 "$OUT/RDREQ.log"; exit 1; }
find "$OUT/RDREQ" -name "*counter_collection.csv" -exec python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Kernel_Name'][:24], r['Counter_Name'], r['Counter_Value'])
" {} \;
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$OUT/$c" -o $c -- scripts/micro/fetch_half > "$OUT/$c.log" 2>&1 || { echo calib $c failed; tail -5 "$OUT/$c.log"; exit 1; }
  find "$OUT/$c" -name "*counter_collection.csv" -exec python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Kernel_Name'][:24], r['Counter_Name'], r['Counter_Value'], 'x1KiB/1GiB', round(float(r['Counter_Value'])*1024/2**30, 4))
" {} \;
done
