#!/bin/bash
# grow tests/golden/dist_c5m.npz in chunks of 32 reference replicas (8 processes, nice 19),
# each chunk appended and saved as it completes; usage: grow_c5m_dist.sh START CHUNKS
cd "$(dirname "$0")/../.."
S=${1:-0}; N=${2:-8}
for k in $(seq 0 $((N - 1))); do
  MPLBACKEND=Agg nice -n 19 python tests/golden/gen_golden.py --c5m-dist 32 --c5m-start $((S + 32 * k)) --procs 8 || exit 1
done
