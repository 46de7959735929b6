#!/bin/bash
# Grow tests/golden/dist_c5s.npz (the reference's own ensemble of graphs.c5_small: C5's
# Hawkes regime at T = 1000 on 4 followers) in chunks at nice 19 until it holds $1
# replicas (default 10000).  CPU only; runs the reference in this container.
set -euo pipefail
cd "$(dirname "$0")/../.."
TARGET=${1:-10000}
PROCS=${PROCS:-2}
CHUNK=${CHUNK:-200}
while true; do
  N=0
  [ -f tests/golden/dist_c5s.npz ] && N=$(python -c "import numpy as np; print(np.load('tests/golden/dist_c5s.npz')['data'].shape[0])")
  [ "$N" -ge "$TARGET" ] && break
  C=$(( TARGET - N < CHUNK ? TARGET - N : CHUNK ))
  echo "$(date +%T) have $N, adding $C" >&2
  nice -n 19 python tests/golden/gen_golden.py --c5s-dist "$C" --c5s-start "$N" --procs "$PROCS"
done
