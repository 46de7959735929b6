set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 400 python3 -u scripts/bench_paths.py > gpurun_out/r04e/paths.json 2> gpurun_out/r04e/paths.err || { tail -20 gpurun_out/r04e/paths.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04e/paths.json'))
for k,v in d.items(): print(k, {a:(round(b,4) if isinstance(b,float) else b) for a,b in v.items() if a!='plan'})
"
for s in replay_batch seq_multigraph_c3 seq_600_sources seq_max_events_c3; do
  scripts/gpu_paths_pmc.sh r04 $s || exit 1
done
