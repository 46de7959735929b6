#!/bin/bash
# A/B: replay workgroup sizes + scan tail loads; then the touched tests on the new build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ab
for so in librq.so librq_rp1024.so librq_rp256.so; do
  RQ_SO_PATH=$PWD/redqueen_amd/$so timeout -k 10 200 python3 -u scripts/dev/ab_replay.py || exit 1
done
for so in librq.so librq_rp1024.so librq.so librq_rp1024.so; do
  RQ_SO_PATH=$PWD/redqueen_amd/$so timeout -k 10 200 python3 -u bench.py --no-cpu --steps 20 > gpurun_out/ab/b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('$so', 'scan_gbs', round(d['scan_gbs']), 'ms', d['kernels_ms_per_launch'], 'step', round(d['ms_per_step'],4))"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_replay_batch.py tests/test_gpu_replay_chunked.py tests/test_gpu_realdata.py tests/test_gpu_stats.py -x -q --timeout 300 --timeout-method thread -p no:logging > gpurun_out/ab/pytest.log 2>&1; tail -2 gpurun_out/ab/pytest.log
