#!/bin/bash
# A/B: scan build waves per SIMD (RQ_SCAN_WPE) on the C3 bench.  usage: ab_scan.sh "2 4 6 8"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ab
for w in ${1:-4 6 8}; do
  RQ_SCAN_WPE=$w timeout -k 10 200 python3 -u bench.py --no-cpu --steps 20 > gpurun_out/ab/s.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/s.json')); print('wpe $w', 'scan_gbs', round(d['scan_gbs']), 'scan_ms', round(d['kernels_ms_per_launch']['scan'],4), 'step', round(d['ms_per_step'],4))"
done
