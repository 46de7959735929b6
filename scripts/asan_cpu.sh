#!/bin/bash
# Host-code sanitizer run: AddressSanitizer + UBSan builds of the CPU
# oracle and of librq's host side, then the CPU test files that drive them through
# ctypes (ABI validation, graph build, the oracle restatements, the facade's host
# logic).  CPU only -- no GPU is touched (the device code is not sanitized).
#   scripts/asan_cpu.sh [extra pytest args]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/oracle" -f asan.mk
make -s -j8 -C "$ROOT/redqueen_amd/csrc" -f asan.mk
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
cd "$ROOT"
# leaks: the interpreter's own allocations are not ours to report
LD_PRELOAD="$RT" \
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:protect_shadow_gap=0 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
RQ_SO_PATH="$ROOT/redqueen_amd/_asan/librq.so" RQO_SO_PATH="$ROOT/oracle/_asan/librq_oracle.so" \
python -m pytest tests/test_abi.py tests/test_oracle.py tests/test_facade_cpu.py tests/test_analysis_cpu.py \
    tests/test_significance_cpu.py -m "not gpu" -q -p no:cacheprovider "$@"
