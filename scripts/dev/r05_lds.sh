set -o pipefail
OUT=gpurun_out/r05lds; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -o "SQ_LDS[A-Z_]*\|SQ_INSTS_LDS\|SQ_INST_CYCLES_VMEM[A-Z_]*\|SQ_INSTS_SMEM[A-Z_]*" $OUT/counters.txt | sort -u | head -30
timeout -k 10 -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/p -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/p.log 2>&1 && echo pmc ok
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt; grep -A12 "^rq_sweep_fwm\|^rq_merge\|^rq_gen" $OUT/summary.txt | head -60
