set -o pipefail
OUT=gpurun_out/r04n; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_batch.py tests/test_gpu_replay_chunked.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; tail -3 $OUT/pytest1.log; [ $rc = 0 ] || exit 1
for v in r2 r3 r2b r3b; do
  so=redqueen_amd/librq.so; case $v in r3*) so=redqueen_amd/librq_r3.so;; esac
  RQ_SO_PATH=$(pwd)/$so timeout -k 10 300 python3 -u scripts/bench_paths.py --only replay_batch,replay_batch_eid,replay_batch_1024 > $OUT/rp_$v.json 2> $OUT/rp_$v.err || { tail -5 $OUT/rp_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/rp_$v.json'))
print('$v', {k:(round(v.get('ms_fast', v.get('ms_replay', 0)),4), round(v.get('GBps',0)), v.get('equal_to_sweep')) for k,v in d.items() if isinstance(v, dict)})"
done
for d in 0 1 2 3; do
  RQ_SWEEP_DBG=$d timeout -k 10 200 python3 -u scripts/c5_phase.py 4096 > $OUT/c5_dbg$d.log 2>&1 || { tail -5 $OUT/c5_dbg$d.log; exit 1; }
  tail -1 $OUT/c5_dbg$d.log
done
scripts/gpu_ab_env.sh r04n --workload c5 --steps 3 -- "pf1=" "pf0=RQ_SO_PATH=$(pwd)/redqueen_amd/librq_pf0.so" "pf1b="
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
