#!/bin/bash
# Sweep diagnostics: per-phase s_memtime split (RQ_PHASE_CLOCK build, librq_clk.so)
# and a host-trap PC-sampling pass over the C3 bench.  usage: scripts/gpu_diag.sh TAG
set -o pipefail
TAG=${1:-diag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
if [ -f redqueen_amd/librq_clk.so ]; then
  RQ_SO_PATH=$ROOT/redqueen_amd/librq_clk.so timeout -k 10 200 python3 scripts/phase_clock.py > "$OUT/clk.log" 2>&1 || { echo "clk failed"; tail -5 "$OUT/clk.log"; exit 1; }
  cat "$OUT/clk.log"
fi
