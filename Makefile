# Top-level build: libcmsbwt.so (HIP, gfx950), the cmsbwt CLI, and the oracle
# (test infrastructure).  Outputs stay in-tree so they travel to the GPU box.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := cms-bwt_amd/csrc
OUT ?= cms-bwt_amd/build
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-function $(XFLAGS)
HOSTFLAGS := -O3 -std=c++17 -fPIC -Wall

# dist_merge.hip is compiled inside engine.hip (one translation unit: the
# engine's rocPRIM instantiations are emitted once, not once per file)
OBJS := $(OUT)/engine.o $(OUT)/multi.o $(OUT)/dist_kernels.o $(OUT)/ms_walk.o $(OUT)/ms_walk2.o $(OUT)/merge.o $(OUT)/synth.o $(OUT)/coll_read.o $(OUT)/ref_index.o $(OUT)/host_index.o $(OUT)/host_reader.o
HDRS := $(wildcard $(SRC)/*.h) include/cmsbwt.h

all: lib cli gen oracle

lib: $(OUT)/libcmsbwt.so
cli: $(OUT)/cmsbwt
gen: $(OUT)/gen_synth

$(OUT):
	mkdir -p $(OUT)

$(OUT)/engine.o: $(SRC)/dist_merge.hip

$(OUT)/%.o: $(SRC)/%.hip $(HDRS) | $(OUT)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# the uniform-step walk keeps its addresses in registers only without
# SimplifyCFG store sinking (which otherwise moves them to scratch), and is
# built without the backend's SIOptimizeVGPRLiveRange pass, which miscompiles
# it (DESIGN.md §3.1 "Round 6": the pass marks the walk's `pos` undefined on a
# path that still reads it; found by tools/memo_isa.sh + opt-bisect)
W2WAVES ?= 4
W2FLAGS := -mllvm -simplifycfg-sink-common=false -mllvm -amdgpu-opt-vgpr-liverange=false
$(OUT)/ms_walk2.o: $(SRC)/ms_walk2.hip $(HDRS) | $(OUT)
	$(HIPCC) $(HIPFLAGS) $(W2FLAGS) -DCMSBWT_W2_WAVES=$(W2WAVES) -c -o $@ $<

$(OUT)/host_%.o: $(SRC)/host_%.cpp $(HDRS) | $(OUT)
	g++ $(HOSTFLAGS) -c -o $@ $<

$(OUT)/libcmsbwt.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS)

$(OUT)/cmsbwt: $(SRC)/cli_main.cpp $(OUT)/libcmsbwt.so include/cmsbwt.h
	g++ $(HOSTFLAGS) -o $@ $< -L$(OUT) -lcmsbwt -Wl,-rpath,'$$ORIGIN'

# synthetic FASTA workload writer, used by bench.py's
# end-to-end leg: product-side, independent of the oracle's copy
$(OUT)/gen_synth: tools/gen_synth.cpp $(SRC)/synth.h | $(OUT)
	g++ $(HOSTFLAGS) -pthread -o $@ tools/gen_synth.cpp

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(OUT)
	$(MAKE) -C oracle clean

.PHONY: all lib cli gen oracle clean
