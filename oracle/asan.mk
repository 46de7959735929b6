# Sanitizer build of the CPU oracle (host code only; test infrastructure):
#   make -f asan.mk     ->  _asan/librq_oracle.so
# clang (ROCm's) so that it shares one ASan runtime with the sanitized librq host code
# (redqueen_amd/csrc/asan.mk); scripts/asan_cpu.sh preloads that runtime into pytest.
CC := /opt/rocm/lib/llvm/bin/clang
SAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-gpu-sanitize -fno-omit-frame-pointer -g
CFLAGS = -O1 -mfma -fPIC -ffp-contract=off -fno-fast-math -Wall $(SAN)

_asan/librq_oracle.so: rq_oracle.c rq_oracle_analysis.c rq_oracle.h ../redqueen_amd/csrc/rq_spec.h ../redqueen_amd/csrc/rq_tables.h
	@mkdir -p _asan
	$(CC) $(CFLAGS) -shared -shared-libsan -o $@ rq_oracle.c rq_oracle_analysis.c -lm -lpthread
