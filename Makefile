# Build of the MI355X-native nonlocal heat-equation solver.
#   libnlh.so   C-ABI solver library (HIP kernels for gfx950 + RCCL)
#   bin/2d_nonlocal_{serial,async,distributed}, bin/1d_nonlocal_serial   drop-in CLI drivers
#   bin/2d_domain_decomposition   --file partition writer (host-only)
#   oracle/liboracle.so   CPU checker (test infrastructure only)
ROCM    ?= /opt/rocm
HIPCC   ?= $(ROCM)/bin/hipcc
ARCH    ?= gfx950
PKG     := nonlocalheatequation_amd
CSRC    := $(PKG)/csrc
LIBDIR  := $(PKG)/lib
OBJDIR  := build/obj
BINDIR  := bin

CXXSTD  := -std=c++17
WARN    := -Wall -Wextra -Wno-unused-parameter
INC     := -Iinclude -I$(CSRC)
HIPFLAGS := --offload-arch=$(ARCH) -O3 $(CXXSTD) -fPIC $(WARN) $(INC) -munsafe-fp-atomics
HOSTFLAGS := -O2 $(CXXSTD) -fPIC $(WARN) $(INC) -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include

# build identity: hash of every library and driver source, the public header
# and this Makefile (flags), in sorted path order --
# nonlocalheatequation_amd.source_build_id() recomputes it from the tree; tests,
# smoke() and bench.py compare the two, and every driver binary checks at start
# that the libnlh it loaded carries the id it was built with
BUILD_ID_SRCS := $(sort $(wildcard $(CSRC)/*.hip $(CSRC)/*.h $(CSRC)/*.cpp $(CSRC)/drivers/*.cpp \
                   $(CSRC)/drivers/*.h) include/nlh.h Makefile)
BUILD_ID := $(shell cat $(BUILD_ID_SRCS) | sha256sum | cut -c1-16)

FAST_UNITS := $(sort $(wildcard $(CSRC)/nlh_fast_e*.hip $(CSRC)/nlh_pair_e*.hip $(CSRC)/nlh_wide_e*.hip))
FAST_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(FAST_UNITS))
LIB_OBJS := $(OBJDIR)/nlh_kernels.o $(FAST_OBJS) $(OBJDIR)/nlh_prefix.o $(OBJDIR)/nlh_api.o $(OBJDIR)/nlh_plan.o \
            $(OBJDIR)/nlh_1d.o
# the fast kernel is fully unrolled over 2E+1 rows; lift LLVM's pragma-unroll
# size cap so every accumulator stays in registers (no scratch)
UNROLL  := -mllvm -pragma-unroll-threshold=1000000
DRIVERS  := $(BINDIR)/2d_nonlocal_serial $(BINDIR)/2d_nonlocal_async $(BINDIR)/2d_nonlocal_distributed \
            $(BINDIR)/1d_nonlocal_serial $(BINDIR)/2d_domain_decomposition $(BINDIR)/comm_id_check
DRV_COMMON := $(OBJDIR)/driver_common.o $(OBJDIR)/vtu_writer.o

all: lib drivers oracle
lib: $(LIBDIR)/libnlh.so
drivers: $(DRIVERS)
oracle:
	$(MAKE) -s -C oracle

$(OBJDIR) $(LIBDIR) $(BINDIR):
	mkdir -p $@

CHDRS := $(CSRC)/nlh_device.h $(CSRC)/nlh_kernel_common.h
KHDRS := $(CHDRS) $(CSRC)/nlh_fast.h $(CSRC)/nlh_pair.h $(CSRC)/nlh_wide.h

$(OBJDIR)/nlh_kernels.o: $(CSRC)/nlh_kernels.hip $(KHDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/nlh_fast_%.o: $(CSRC)/nlh_fast_%.hip $(CHDRS) $(CSRC)/nlh_fast.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(UNROLL) -c $< -o $@

$(OBJDIR)/nlh_pair_%.o: $(CSRC)/nlh_pair_%.hip $(CHDRS) $(CSRC)/nlh_pair.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(UNROLL) -c $< -o $@

$(OBJDIR)/nlh_wide_%.o: $(CSRC)/nlh_wide_%.hip $(CHDRS) $(CSRC)/nlh_wide.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(UNROLL) -c $< -o $@

$(OBJDIR)/nlh_prefix.o: $(CSRC)/nlh_prefix.hip $(CHDRS) $(CSRC)/nlh_prefix.h $(CSRC)/nlh_rt.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/nlh_api.o: $(CSRC)/nlh_api.cpp $(BUILD_ID_SRCS) | $(OBJDIR)
	$(HIPCC) $(HOSTFLAGS) -DNLH_BUILD_ID='"$(BUILD_ID)"' -x c++ -c $< -o $@

$(OBJDIR)/nlh_1d.o: $(CSRC)/nlh_1d.cpp include/nlh.h | $(OBJDIR)
	$(HIPCC) $(HOSTFLAGS) -x c++ -c $< -o $@

$(OBJDIR)/nlh_plan.o: $(CSRC)/nlh_plan.cpp $(CSRC)/nlh_plan.h | $(OBJDIR)
	g++ $(HOSTFLAGS) -c $< -o $@

$(LIBDIR)/libnlh.so: $(LIB_OBJS) | $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(LIB_OBJS) -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib

$(OBJDIR)/driver_common.o: $(CSRC)/drivers/driver_common.cpp $(BUILD_ID_SRCS) | $(OBJDIR)
	g++ -O2 $(CXXSTD) $(WARN) $(INC) -DNLH_DRIVER_BUILD_ID='"$(BUILD_ID)"' -c $< -o $@

$(OBJDIR)/vtu_writer.o: $(CSRC)/drivers/vtu_writer.cpp $(CSRC)/drivers/vtu_writer.h | $(OBJDIR)
	g++ -O2 $(CXXSTD) $(WARN) $(INC) -c $< -o $@

$(BINDIR)/%: $(CSRC)/drivers/%.cpp $(DRV_COMMON) $(LIBDIR)/libnlh.so | $(BINDIR)
	g++ -O2 $(CXXSTD) $(WARN) $(INC) $< $(DRV_COMMON) -o $@ -L$(LIBDIR) -lnlh \
	    -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,$(ROCM)/lib -lpthread

# test harness of the drivers' TCP id bootstrap (tests/test_drivers.py, CPU)
$(BINDIR)/comm_id_check: tools/comm_id_check.cpp $(DRV_COMMON) $(LIBDIR)/libnlh.so | $(BINDIR)
	g++ -O2 $(CXXSTD) $(WARN) $(INC) -I$(CSRC)/drivers $< $(DRV_COMMON) -o $@ -L$(LIBDIR) -lnlh \
	    -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' -Wl,-rpath,$(ROCM)/lib -lpthread

clean:
	rm -rf build $(LIBDIR) $(BINDIR)
	$(MAKE) -s -C oracle clean

.PHONY: all lib drivers oracle clean
