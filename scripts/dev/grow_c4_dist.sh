#!/bin/bash
# Grow tests/golden/dist_c4.npz (the reference's own ensembles at the six C4 corners)
# in chunks, at nice 19, until it holds $1 replicas per point (default 10000).
# CPU only; runs the reference in this container.
set -euo pipefail
cd "$(dirname "$0")/../.."
TARGET=${1:-10000}
PROCS=${PROCS:-6}
CHUNK=${CHUNK:-2000}
while true; do
  N=$(python -c "import numpy as np, os; p='tests/golden/dist_c4.npz'; print(np.load(p)['data'].shape[1] if os.path.exists(p) else 0)")
  [ "$N" -ge "$TARGET" ] && break
  C=$(( TARGET - N < CHUNK ? TARGET - N : CHUNK ))
  echo "$(date +%T) have $N, adding $C" >&2
  nice -n 19 python tests/golden/gen_golden.py --c4-dist "$C" --c4-start "$N" --procs "$PROCS"
done
