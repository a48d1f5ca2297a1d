# Top-level build. `make` builds everything in-tree (the .so files travel to the
# GPU box with the gpurun snapshot). gfx950 only.
HIPCC   ?= /opt/rocm/bin/hipcc
CLANGXX ?= /opt/rocm/llvm/bin/clang++
ARCH    ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function
CSRC := bdls_amd/csrc
LIB  := bdls_amd/lib

HDRS := $(wildcard $(CSRC)/*.h) include/bdls_hip.h

all: $(LIB)/libbdlship.so $(LIB)/libbdlsgen.so oracle tests/native/build/libhostsim.so $(LIB)/csp_load

$(LIB)/verify_kernels.o: $(CSRC)/verify_kernels.hip $(HDRS)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB)/bdls_hip.o: $(CSRC)/bdls_hip.cpp $(HDRS)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB)/bdls_msg.o: $(CSRC)/bdls_msg.cpp include/bdls_hip.h
	@mkdir -p $(LIB)
	g++ -O2 -std=c++17 -fPIC -Wall -c $< -o $@

$(LIB)/fabric.o: $(CSRC)/fabric.cpp $(HDRS)
	@mkdir -p $(LIB)
	g++ -O2 -std=c++17 -fPIC -Wall -Wno-unknown-pragmas -c $< -o $@

$(LIB)/libbdlship.so: $(LIB)/verify_kernels.o $(LIB)/bdls_hip.o $(LIB)/bdls_msg.o $(LIB)/fabric.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lpthread

$(LIB)/libbdlsgen.so: bdls_amd/workload/gen.c
	@mkdir -p $(LIB)
	gcc -O2 -fPIC -shared -Wall -o $@ $< -lcrypto -lpthread

oracle:
	$(MAKE) -C oracle

# test-only host build of the device arithmetic (never linked into the product)
tests/native/build/libhostsim.so: tests/native/hostsim.cpp $(HDRS)
	@mkdir -p tests/native/build
	$(CLANGXX) -O2 -std=c++17 -shared -fPIC -o $@ $< -lpthread

# build-kernel experiments (profiles/r02/exp_build): not part of `all`
EXP_VARIANTS := base:
exp:
	@mkdir -p build/exp
	@for v in $(EXP_VARIANTS); do n=$${v%%:*}; f=$$(echo $${v#*:} | tr '+' ' '); \
	  $(HIPCC) $(HIPFLAGS) $$f -c $(CSRC)/verify_kernels.hip -o build/exp/vk_$$n.o && \
	  $(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/exp/libbdlship_$$n.so build/exp/vk_$$n.o \
	    $(LIB)/bdls_hip.o $(LIB)/bdls_msg.o $(LIB)/fabric.o -lpthread || exit 1; done

clean:
	rm -rf $(LIB) tests/native/build
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

$(LIB)/ubench: $(CSRC)/ubench.hip $(HDRS)
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) -o $@ $<
all: $(LIB)/ubench

# native load generator for the coalesced single Verify (bench.py side configs)
$(LIB)/csp_load: tools/csp_load.cpp include/bdls_hip.h $(LIB)/libbdlship.so
	g++ -O2 -std=c++17 -Wall -o $@ $< -L$(LIB) -lbdlship -Wl,-rpath,'$$ORIGIN' -lpthread
