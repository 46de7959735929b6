set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_merge.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest1.log 2>&1; rc=$?; tail -3 $OUT/pytest1.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 -u scripts/bench_paths.py --only seq_600_sources,fast_600_sources,fast_3000_sources > $OUT/paths.json 2> $OUT/paths.err || { tail -5 $OUT/paths.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/paths.json'))
for k,v in d.items(): print(k, {a:(round(b,4) if isinstance(b,float) else b) for a,b in v.items() if a!='plan'})"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit 1
scripts/gpu_ab_env.sh r04l -- "c3=" && scripts/gpu_ab_env.sh r04l --workload c5 --steps 4 -- "c5="
