# Build recipes.  `make` builds everything that ships to the GPU box:
#   whisper-git_amd/wgraph/libwgraph.so   the HIP engine (gfx950) + C ABI
#   whisper-git_amd/wgraph/libwgsynth.so  synthetic DAG generator (workload)
#   oracle/liboracle.so                   CPU oracle (test infrastructure)
#   profiles/microbench/store_ceiling     16-B store bandwidth ceiling (roofline context)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := whisper-git_amd
CSRC    := $(PKG)/csrc
HIPSRC  := $(wildcard $(CSRC)/*.hip)
HIPHDR  := $(wildcard $(CSRC)/*.h) include/wgraph.h include/wgraph_tess.h
# Bit-exact f32: no FMA contraction, IEEE denormals, correctly rounded div/sqrt.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt \
            -Wall -Wno-unused-function -Iinclude -I$(CSRC)
CFLAGS_ORACLE := -O2 -std=c11 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function

all: $(PKG)/wgraph/libwgraph.so $(PKG)/wgraph/libwgsynth.so oracle/liboracle.so profiles/microbench/store_ceiling

$(PKG)/wgraph/libwgraph.so: $(HIPSRC) $(HIPHDR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIPSRC)

$(PKG)/wgraph/libwgsynth.so: $(PKG)/synth/wg_synth.c
	gcc -O2 -std=c11 -fPIC -shared -Wall -o $@ $< -lm

oracle/liboracle.so: oracle/wg_oracle.c include/wgraph.h include/wgraph_tess.h
	gcc $(CFLAGS_ORACLE) -shared -o $@ oracle/wg_oracle.c -lm

profiles/microbench/store_ceiling: profiles/microbench/store_ceiling.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

oracle: oracle/liboracle.so
synth: $(PKG)/wgraph/libwgsynth.so
engine: $(PKG)/wgraph/libwgraph.so

clean:
	rm -f $(PKG)/wgraph/*.so oracle/*.so profiles/microbench/store_ceiling

.PHONY: all clean oracle synth engine
