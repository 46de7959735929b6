# Sanitizer build of librq's HOST code (graph build, plan, workspace / ABI validation,
# the pinned staging ring): every -fsanitize applies to the host compilation only
# (-Xarch_host); the gfx950 device code is the normal build.
#   make -f asan.mk     ->  ../_asan/librq.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HSAN = -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
       -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer
FLAGS = -O2 -g --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -fPIC -std=c++17 $(HSAN)
OUT = ../_asan/librq.so
BUILD = build_asan
SRC = rq_kernels.hip rq_sweep_fw.hip rq_merge.hip rq_analysis.hip rq_replay.hip rq_api.cpp
OBJ = $(addprefix $(BUILD)/,$(addsuffix .o,$(SRC)))
HDR = rq_spec.h rq_tables.h rq_device.h rq_internal.h rq_gen.h rq_sweep_core.h ../../include/rq.h

$(OUT): $(OBJ)
	@mkdir -p ../_asan
	$(HIPCC) --offload-arch=$(ARCH) -shared -Xarch_host -shared-libsan $(HSAN) -o $@ $(OBJ)

$(BUILD)/%.o: % $(HDR)
	@mkdir -p $(BUILD)
	$(HIPCC) $(FLAGS) -c -o $@ $<
