# Build of the MI355X-native AnySeq engine (gfx950) and the CPU oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-parameter
SRC := anyseq_amd/csrc
LIB := anyseq_amd/libanyseq.so

all: $(LIB) oracle

# the steady-state loop of the fill kernel is generated asm (tools/gen_block_asm.py)
$(SRC)/anyseq_block_asm.inc: tools/gen_block_asm.py
	python3 tools/gen_block_asm.py > /dev/null

$(SRC)/anyseq_kernels.o: $(SRC)/anyseq_kernels.hip $(SRC)/anyseq_internal.h $(SRC)/anyseq_block_asm.inc
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -c $< -o $@

$(SRC)/anyseq_engine.o: $(SRC)/anyseq_engine.cpp $(SRC)/anyseq_internal.h $(SRC)/anyseq_host.h include/anyseq.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/anyseq_shard.o: $(SRC)/anyseq_shard.cpp $(SRC)/anyseq_internal.h $(SRC)/anyseq_host.h include/anyseq.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/anyseq_io.o: $(SRC)/anyseq_io.cpp include/anyseq.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/anyseq_aux.o: $(SRC)/anyseq_aux.hip $(SRC)/anyseq_internal.h
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -c $< -o $@

$(LIB): $(SRC)/anyseq_kernels.o $(SRC)/anyseq_engine.o $(SRC)/anyseq_shard.o $(SRC)/anyseq_io.o $(SRC)/anyseq_aux.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -Wl,-z,defs -o $@ $^ -L/opt/rocm/lib -lrccl -lhsa-runtime64

oracle:
	$(MAKE) -s -C oracle

# diagnostic build with s_memtime stamps (tools only; never loaded by the product path)
stamps: anyseq_amd/libanyseq_stamps.so
anyseq_amd/libanyseq_stamps.so: $(SRC)/anyseq_kernels.hip $(SRC)/anyseq_engine.o $(SRC)/anyseq_shard.o $(SRC)/anyseq_io.o $(SRC)/anyseq_aux.o $(SRC)/anyseq_internal.h $(SRC)/anyseq_block_asm.inc
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -DANYSEQ_STAMPS -c $(SRC)/anyseq_kernels.hip -o $(SRC)/anyseq_kernels_stamps.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(SRC)/anyseq_kernels_stamps.o $(SRC)/anyseq_engine.o $(SRC)/anyseq_shard.o $(SRC)/anyseq_io.o $(SRC)/anyseq_aux.o -L/opt/rocm/lib -lrccl -lhsa-runtime64

# experimental build for A/B runs: the affine loop generated under other generator knobs
# (EXPGEN, e.g. `make exp EXPGEN="ANYSEQ_GEN_LEAN=0"`) as anyseq_amd/libanyseq_exp.so,
# loaded with ANYSEQ_LIB
# (EXPDEF: extra -D flags of the kernels, e.g. EXPGEN="ANYSEQ_GEN_GS=0" EXPDEF=-DANYSEQ_AFF_GS=0)
EXPGEN ?= ANYSEQ_GEN_LEAN=1
EXPDEF ?=
exp:
	mkdir -p build && env $(EXPGEN) python3 tools/gen_block_asm.py build/exp_asm.inc > /dev/null
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) $(EXPDEF) -DANYSEQ_ASM_INC='"$(CURDIR)/build/exp_asm.inc"' -c $(SRC)/anyseq_kernels.hip -o build/anyseq_kernels_exp.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -Wl,-z,defs -o anyseq_amd/libanyseq_exp.so build/anyseq_kernels_exp.o $(SRC)/anyseq_engine.o $(SRC)/anyseq_shard.o $(SRC)/anyseq_io.o $(SRC)/anyseq_aux.o -L/opt/rocm/lib -lrccl -lhsa-runtime64

# diagnostic build with only the steady-state stamps (band lags at a product-like step)
stamps_light:
	mkdir -p build && ANYSEQ_GEN_TSLIGHT=1 python3 tools/gen_block_asm.py build/light_asm.inc > /dev/null
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -DANYSEQ_STAMPS -DANYSEQ_ASM_INC='"$(CURDIR)/build/light_asm.inc"' -c $(SRC)/anyseq_kernels.hip -o build/anyseq_kernels_light.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o anyseq_amd/libanyseq_stamps_light.so build/anyseq_kernels_light.o $(SRC)/anyseq_engine.o $(SRC)/anyseq_shard.o $(SRC)/anyseq_io.o $(SRC)/anyseq_aux.o -L/opt/rocm/lib -lrccl -lhsa-runtime64

clean:
	rm -f $(SRC)/*.o $(LIB) anyseq_amd/libanyseq_*.so
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean stamps exp stamps_light
