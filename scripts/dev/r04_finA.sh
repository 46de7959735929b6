set -o pipefail
bash scripts/gpu_round.sh r04fin && bash scripts/gpu_pmc.sh r04c3 c3 10000
