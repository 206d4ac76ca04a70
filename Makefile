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
SRCS     := $(CSRC)/stream_pass.hip $(CSRC)/gram.hip $(CSRC)/resident.hip $(CSRC)/coordinate.hip $(CSRC)/weiszfeld.hip $(CSRC)/oma.hip $(CSRC)/pack.hip $(CSRC)/clients.hip $(CSRC)/api.hip
OBJS     := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(SRCS))
HDRS     := $(wildcard $(CSRC)/*.h) include/gmagg.h

all: $(LIB)

# gram.hip without SLP vectorization: the f16 Gram producer's per-element FMAs stay
# scalar v_fma_f32 instead of v_pk_fma_f32, which the MFMA waves sharing its SIMD pay
# for (C4 shard Gram partial 3.30 -> 2.97 ms; profiles/r2_gram_producer_ab.txt)
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

# A/B build: the streaming pass with the two-tile PIPE schedule compiled in
# (GMAGG_PASS_VARIANT=1 selects it; GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so
# loads this library at run time).
ALT := byzantine_aircomp_amd/libgmagg_alt.so
$(BUILD)/alt/stream_pass.o: $(CSRC)/stream_pass.hip $(HDRS)
	@mkdir -p $(BUILD)/alt
	$(HIPCC) $(HIPFLAGS) -DGMK_PIPE_VARIANT -c $< -o $@
$(ALT): $(BUILD)/alt/stream_pass.o $(filter-out $(BUILD)/stream_pass.o,$(OBJS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lrccl \
	    -Wl,-rpath,/opt/rocm/lib
alt: $(ALT)
.PHONY: alt
