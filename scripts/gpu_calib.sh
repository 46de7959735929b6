#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (scripts/micro/fetch_calib) on the GPU box.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-calib}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/f" -o f -- scripts/micro/fetch_calib > "$OUT/f.log" 2>&1 || { echo calib failed; tail -5 "$OUT/f.log"; exit 1; }
find "$OUT/f" -name "*counter_collection.csv" -exec python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Kernel_Name'][:40], r['Counter_Name'], r['Counter_Value'], 'ratio_vs_1GiB', float(r['Counter_Value'])*1024/2**30)
" {} \;
