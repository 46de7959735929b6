#!/bin/bash
# A/B of alternative librq builds (RQ_SO_PATH) on the C3 bench.  usage: ab_so.sh "librq.so librq_x.so ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ab
for so in $1; do
  RQ_SO_PATH=$PWD/redqueen_amd/$so timeout -k 10 200 python3 -u bench.py --no-cpu --steps 20 > gpurun_out/ab/so.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/so.json')); k=d['kernels_ms_per_launch']; print('$so', 'merge', round(k['merge_streams'],4), 'sweep', round(k['sweep'],4), 'step', round(d['ms_per_step'],4), round(d['value']))"
done
