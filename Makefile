# Build the MI355X (gfx950) aggregation library and the CPU oracle helpers.
#   make            -> byzantine_aircomp_amd/libgmagg.so
#   make clean
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC     := byzantine_aircomp_amd/csrc
BUILD    := build/obj
LIB      := byzantine_aircomp_amd/libgmagg.so
HIPFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-result \
            -I include -munsafe-fp-atomics
SRCS     := $(CSRC)/stream_pass.hip $(CSRC)/gram.hip $(CSRC)/resident.hip $(CSRC)/resident_batched.hip $(CSRC)/coordinate.hip $(CSRC)/weiszfeld.hip $(CSRC)/oma.hip $(CSRC)/pack.hip $(CSRC)/clients.hip $(CSRC)/api.hip $(CSRC)/rows_pass.hip
OBJS     := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(SRCS))
HDRS     := $(wildcard $(CSRC)/*.h) include/gmagg.h

all: $(LIB)

# gram.hip without SLP vectorization: the f16 Gram producer's per-element FMAs stay
# scalar v_fma_f32 instead of v_pk_fma_f32, which the MFMA waves sharing its SIMD pay
# for (C4 shard Gram partial 3.30 -> 2.97 ms; profiles/history/r2_gram_producer_ab.txt)
$(BUILD)/gram.o: HIPFLAGS += -fno-slp-vectorize

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -L/opt/rocm/lib -lrccl \
	    -Wl,-rpath,/opt/rocm/lib

clean:
	rm -rf $(BUILD) $(LIB)

.PHONY: all clean

# A/B build: every object compiled again with ALT_FLAGS into build/alt, linked as
# byzantine_aircomp_amd/libgmagg_alt.so; GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so
# loads it at run time (tools/ab.py --variant alt=GMAGG_LIB=...).
#   make alt ALT_FLAGS=-DGMK_H16_SHAPE=16
# ALT_ONLY="resident resident_batched": recompile only those sources with ALT_FLAGS and
# link the product's objects for the rest (the flags' macros live in those files).
ALT       := byzantine_aircomp_amd/libgmagg_alt.so
ALT_FLAGS ?= -DGMK_PIPE_VARIANT
ALT_ONLY  ?=
ALT_SEL   := $(if $(ALT_ONLY),$(foreach n,$(ALT_ONLY),$(CSRC)/$(n).hip),$(SRCS))
ALT_OBJS  := $(patsubst $(CSRC)/%.hip,$(BUILD)/alt/%.o,$(ALT_SEL)) \
             $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(filter-out $(ALT_SEL),$(SRCS)))
$(BUILD)/alt/gram.o: HIPFLAGS += -fno-slp-vectorize
$(BUILD)/alt/%.o: $(CSRC)/%.hip $(HDRS) FORCE
	@mkdir -p $(BUILD)/alt
	$(HIPCC) $(HIPFLAGS) $(ALT_FLAGS) -c $< -o $@
$(ALT): $(ALT_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(ALT_OBJS) -L/opt/rocm/lib -lrccl \
	    -Wl,-rpath,/opt/rocm/lib
alt: $(ALT)
FORCE:
.PHONY: alt FORCE
