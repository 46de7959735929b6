#!/bin/bash
# Grow tests/golden/dist_c3.npz (the reference's own C3 ensemble) in chunks, at
# nice 19, until the file holds $1 replicas (default 10000).  Each chunk appends
# CHUNK replicas through gen_golden.py --c3-dist/--c3-start, so an interrupted run
# keeps every finished chunk.  CPU only; runs the reference in this container.
set -euo pipefail
cd "$(dirname "$0")/../.."
TARGET=${1:-10000}
PROCS=${PROCS:-7}
CHUNK=${CHUNK:-56}
while true; do
  N=$(python -c "import numpy as np; print(np.load('tests/golden/dist_c3.npz')['data'].shape[0])")
  [ "$N" -ge "$TARGET" ] && break
  C=$(( TARGET - N < CHUNK ? TARGET - N : CHUNK ))
  echo "$(date +%T) have $N, adding $C" >&2
  nice -n 19 python tests/golden/gen_golden.py --c3-dist "$C" --c3-start "$N" --procs "$PROCS"
done
