set -o pipefail
OUT=gpurun_out/r04paths; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/bench_paths.py > $OUT/paths.json 2> $OUT/paths.err || { tail -20 $OUT/paths.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/paths.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a:(round(b,4) if isinstance(b,float) else b) for a,b in v.items() if a!='plan'})"
bash scripts/gpu_paths_pmc.sh r04 replay_batch && bash scripts/gpu_paths_pmc.sh r04 replay_batch_1024 && bash scripts/gpu_paths_pmc.sh r04 fast_600_sources
