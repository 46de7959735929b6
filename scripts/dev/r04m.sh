set -o pipefail
OUT=gpurun_out/r04m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_merge.py tests/test_gpu_replay.py tests/test_gpu_replay_batch.py tests/test_gpu_replay_chunked.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; tail -3 $OUT/pytest1.log; [ $rc = 0 ] || exit 1
for v in r2 r1 r2b; do
  so=redqueen_amd/librq.so; [ $v = r1 ] && so=redqueen_amd/librq_r1.so
  RQ_SO_PATH=$(pwd)/$so timeout -k 10 300 python3 -u scripts/bench_paths.py --only replay_batch,replay_batch_eid,replay_batch_1024,replay_one_df,replay_one_df_one_workgroup > $OUT/rp_$v.json 2> $OUT/rp_$v.err || { tail -5 $OUT/rp_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/rp_$v.json'))
print('$v', {k:(round(v.get('ms_fast', v.get('ms_replay', 0)),4), round(v.get('GBps',0)), v.get('equal_to_sweep')) for k,v in d.items() if isinstance(v, dict)})"
done
timeout -k 10 300 python3 -u scripts/bench_paths.py --only seq_600_sources,fast_600_sources,fast_3000_sources > $OUT/paths.json 2> $OUT/paths.err || { tail -5 $OUT/paths.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/paths.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a:(round(b,4) if isinstance(b,float) else b) for a,b in v.items() if a!='plan'})"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04m -- "c3=" && scripts/gpu_ab_env.sh r04m --workload c5 --steps 4 -- "c5="
