set -o pipefail
for i in 1 2; do for L in redqueen_amd/librq_base.so redqueen_amd/librq.so; do
RQ_SO_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python3 scripts/bench_paths.py --only fast_600_sources,fast_3000_sources > gpurun_out/ab600.json 2>gpurun_out/ab600.err || { tail -3 gpurun_out/ab600.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab600.json')); print('$L', {k: round(v.get('replicas_per_s',0)) for k,v in d.items() if isinstance(v, dict)})"
done; done
