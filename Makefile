# Top-level build: the HIP product library, the `sahara` CLI and the oracle.
# gfx950 (MI355X) only. `make -j8` here cross-compiles without a GPU.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall
LIBDIR   := sahara_amd/lib
OBJDIR   := build/obj
CSRC     := sahara_amd/csrc
LIB      := $(LIBDIR)/libsahara_hip.so
CLI      := bin/sahara
HDRS     := $(wildcard $(CSRC)/*.h) include/sahara_hip.h

# the build id compiled into the library (tools/build_id.py: a hash of the
# sources); the header is rewritten only when the id changes
BUILD_ID := $(shell python3 tools/build_id.py)
$(shell mkdir -p $(OBJDIR) && echo '#define SAHARA_BUILD_ID "$(BUILD_ID)"' > $(OBJDIR)/build_id.h.new && \
        (cmp -s $(OBJDIR)/build_id.h.new $(OBJDIR)/build_id.h || mv $(OBJDIR)/build_id.h.new $(OBJDIR)/build_id.h))

OBJS := $(OBJDIR)/index_build.o $(OBJDIR)/search.o $(OBJDIR)/capi.o $(OBJDIR)/staging.o $(OBJDIR)/pass.o \
        $(OBJDIR)/host_util.o $(OBJDIR)/scheme.o

all: $(LIB) oracle $(if $(wildcard sahara_amd/cli/*.cpp),$(CLI),) tools/gather_bench

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/capi.o: $(OBJDIR)/build_id.h
$(OBJDIR)/capi.o: HIPFLAGS += -include $(OBJDIR)/build_id.h

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@ -lpthread

CLI_SRC := $(wildcard sahara_amd/cli/*.cpp)
$(CLI): $(CLI_SRC) $(wildcard sahara_amd/cli/*.h) include/sahara_hip.h $(LIB)
	@mkdir -p bin
	g++ $(CXXFLAGS) -Iinclude $(CLI_SRC) -o $@ -L$(LIBDIR) -lsahara_hip -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

tools/gather_bench: tools/gather_bench.hip
	$(HIPCC) $(HIPFLAGS) $< -o $@

oracle:
	$(MAKE) -C oracle

# Host sanitizer builds: AddressSanitizer + UBSan on the host code
# only (no GPU sanitizer on this pool). tools/asan_cpu_tests.sh runs the CPU
# test suite against them.
ASAN_HOST := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer
ASANDIR   := build/asan
ASAN_OBJS := $(ASANDIR)/index_build.o $(ASANDIR)/search.o $(ASANDIR)/capi.o $(ASANDIR)/staging.o $(ASANDIR)/pass.o \
             $(ASANDIR)/host_util.o $(ASANDIR)/scheme.o

$(ASANDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(ASANDIR)
	$(HIPCC) $(HIPFLAGS) -O1 $(ASAN_HOST) -c $< -o $@

$(ASANDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(ASANDIR)
	$(HIPCC) $(HIPFLAGS) -O1 $(ASAN_HOST) -c $< -o $@

$(ASANDIR)/capi.o: $(OBJDIR)/build_id.h
$(ASANDIR)/capi.o: HIPFLAGS += -include $(OBJDIR)/build_id.h

$(ASANDIR)/libsahara_hip.so: $(ASAN_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(ASAN_OBJS) -o $@ -lpthread

bin/sahara_asan: $(CLI_SRC) $(wildcard sahara_amd/cli/*.h) include/sahara_hip.h $(LIB)
	@mkdir -p bin
	g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -Iinclude $(CLI_SRC) -o $@ \
	    -L$(LIBDIR) -lsahara_hip -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -lpthread

asan: $(ASANDIR)/libsahara_hip.so bin/sahara_asan
	$(MAKE) -C oracle asan

clean:
	rm -rf build $(LIBDIR) bin
	$(MAKE) -C oracle clean

.PHONY: all clean oracle asan
