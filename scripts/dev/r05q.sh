# replay A/B (librq_base = round-5 stamped build) + the phase clock of the current source
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_batch.py tests/test_gpu_replay_chunked.py tests/test_gpu_realdata.py tests/test_gpu_analysis.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for L in ${LIBS:-librq_base.so librq.so librq_base.so librq.so}; do
  RQ_SO_PATH=$PWD/redqueen_amd/$L timeout -k 10 300 python3 scripts/bench_paths.py --only ${SECS:-replay_batch,replay_batch_1024} > $O/bp.json 2> $O/bp.err || { tail -5 $O/bp.err; exit 1; }
  python3 scripts/dev/bp_summary.py $O/bp.json $L
done
[ -n "$NOCLK" ] || RQ_SO_PATH=$PWD/redqueen_amd/librq_clk.so timeout -k 10 300 python3 scripts/dev/replay_clock.py
