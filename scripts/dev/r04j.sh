set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_merge.py tests/test_gpu_configs.py tests/test_gpu_graphs.py tests/test_gpu_policy.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04j -- "c3=" || exit 1
for v in "c5_4096:--replicas 4096:" "c5_8192:--replicas 8192:" "c5_8192p1:--replicas 8192:RQ_PIPE=1" "c5_8192p1o0:--replicas 8192:RQ_PIPE=1 RQ_ORDER=0"; do
  n=${v%%:*}; r=${v#*:}; e=${r#*:}; r=${r%%:*}
  env $e timeout -k 10 300 python3 -u bench.py --workload c5 --steps 4 --warmup 2 --no-cpu $r > $OUT/$n.log 2>&1 || { echo $n failed; tail -5 $OUT/$n.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$OUT/$n.log').read().strip().splitlines()[-1]); print('$n', round(l['value']), round(l['ms_per_step'],2), {k: round(v,2) for k,v in l['kernels_ms_per_launch'].items()}, l['sweep_plan']['chunk'], l['overflow'])"
done
