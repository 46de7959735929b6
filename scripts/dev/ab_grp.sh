# merge group size A/B (RQ_MG_GRP=512: the round-5 groups) on the > 512-source paths
set -o pipefail
for i in 1 2; do for G in 512 64; do
RQ_MG_GRP=$G timeout -k 10 200 python3 scripts/bench_paths.py --only fast_600_sources,fast_3000_sources,seq_600_sources > gpurun_out/abg.json 2>gpurun_out/abg.err || { tail -3 gpurun_out/abg.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/abg.json')); print('grp $G', {k: round(v.get('replicas_per_s',0)) for k,v in d.items() if isinstance(v, dict)})"
done; done
