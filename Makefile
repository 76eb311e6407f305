# Build recipes.  `make` builds everything that ships to the GPU box:
#   whisper-git_amd/wgraph/libwgraph.so   the HIP engine (gfx950) + C ABI
#   whisper-git_amd/wgraph/libwgsynth.so  synthetic DAG generator (workload)
#   whisper-git_amd/wgraph/libwgraph_host.so  C++ GraphLayout mirror over the C ABI
#   oracle/liboracle.so                   CPU oracle (test infrastructure)
#   tests/cpp/test_graph_layout           C++ tests of the mirror (engine vs oracle)
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
CXXFLAGS_HOST := -O2 -std=c++17 -fPIC -Wall -Wextra -Iinclude
# The oracle doubles as bench.py's single-thread CPU baseline: -O3 with the
# x86-64-v3 ISA (AVX2/BMI2), not -march=native — it is built in this container
# and runs on the GPU box's host, whose CPU model differs.  No FMA contraction.
CFLAGS_ORACLE := -O3 -march=x86-64-v3 -std=c11 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function

all: $(PKG)/wgraph/libwgraph.so $(PKG)/wgraph/libwgraph_host.so $(PKG)/wgraph/libwgsynth.so oracle/liboracle.so oracle/libedt_cpu.so oracle/libcpu_mt.so \
     tests/cpp/test_graph_layout profiles/microbench/store_ceiling profiles/microbench/store_sweep profiles/microbench/store_align profiles/microbench/launch_cost

# one object per source (parallel, incremental); device code is per translation
# unit (no relocatable device code), host code links into one library
HIPOBJ  := $(patsubst $(CSRC)/%.hip,build/obj/%.o,$(HIPSRC))
build/obj/%.o: $(CSRC)/%.hip $(HIPHDR)
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(PKG)/wgraph/libwgraph.so: $(HIPOBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIPOBJ)

$(PKG)/wgraph/libwgraph_host.so: $(PKG)/host/graph_layout.cpp $(PKG)/host/graph_layout.hpp include/wgraph.h $(PKG)/wgraph/libwgraph.so
	g++ $(CXXFLAGS_HOST) -shared -o $@ $(PKG)/host/graph_layout.cpp -L$(PKG)/wgraph -lwgraph -Wl,-rpath,'$$ORIGIN'

tests/cpp/test_graph_layout: tests/cpp/test_graph_layout.cpp $(PKG)/host/graph_layout.hpp oracle/wg_oracle.h \
                             $(PKG)/synth/wg_synth.h $(PKG)/wgraph/libwgraph_host.so oracle/liboracle.so $(PKG)/wgraph/libwgsynth.so
	g++ $(CXXFLAGS_HOST) -I$(PKG)/host -Ioracle -I$(PKG)/synth -o $@ tests/cpp/test_graph_layout.cpp \
	    -L$(PKG)/wgraph -lwgraph_host -lwgraph -lwgsynth -Loracle -loracle \
	    -Wl,-rpath,'$$ORIGIN/../../$(PKG)/wgraph' -Wl,-rpath,'$$ORIGIN/../../oracle'

$(PKG)/wgraph/libwgsynth.so: $(PKG)/synth/wg_synth.c $(PKG)/synth/wg_synth.h
	gcc -O2 -std=c11 -fPIC -shared -Wall -o $@ $< -lm

oracle/liboracle.so: oracle/wg_oracle.c oracle/wg_oracle.h include/wgraph.h include/wgraph_tess.h
	gcc $(CFLAGS_ORACLE) -shared -o $@ oracle/wg_oracle.c -lm

profiles/microbench/store_ceiling: profiles/microbench/store_ceiling.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

profiles/microbench/store_sweep: profiles/microbench/store_sweep.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

profiles/microbench/store_align: profiles/microbench/store_align.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

profiles/microbench/launch_cost: profiles/microbench/launch_cost.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Wno-unused-value -Wno-unused-result -o $@ $<

# C2's CPU leg (bench.py): exact Felzenszwalb-Huttenlocher EDT, OpenMP
oracle/libedt_cpu.so: oracle/edt_cpu.c
	gcc $(CFLAGS_ORACLE) -fopenmp -shared -o $@ $< -lm

# bench.py's multi-threaded CPU baseline (cpu_baseline_threads): OpenMP port, bit-exact with the oracle
oracle/libcpu_mt.so: oracle/cpu_mt.c oracle/wg_oracle.h include/wgraph.h include/wgraph_tess.h
	gcc $(CFLAGS_ORACLE) -fopenmp -shared -o $@ oracle/cpu_mt.c -lm

oracle: oracle/liboracle.so oracle/libedt_cpu.so oracle/libcpu_mt.so
synth: $(PKG)/wgraph/libwgsynth.so
engine: $(PKG)/wgraph/libwgraph.so
host: $(PKG)/wgraph/libwgraph_host.so tests/cpp/test_graph_layout

clean:
	rm -rf build/obj; rm -f $(PKG)/wgraph/*.so oracle/*.so profiles/microbench/store_ceiling profiles/microbench/store_sweep profiles/microbench/store_align profiles/microbench/launch_cost tests/cpp/test_graph_layout

.PHONY: all clean oracle synth engine host
