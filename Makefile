# Top-level build: the product library (HIP, gfx950) and the oracle (gcc, test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := gnss_sim_receiver_amd
CSRC := $(PKG)/csrc
HIP_SRCS := $(wildcard $(CSRC)/*.hip)
CPP_SRCS := $(wildcard $(CSRC)/*.cpp)
HDRS := $(wildcard $(CSRC)/*.h) include/gnsship.h
# -ffp-contract=off: no implicit fusion anywhere (the HIP header intrinsics __fmul_rn/__fadd_rn
# carry contract flags and were fused into v_fma_f32 otherwise, breaking the bit-exact chip index);
# fused multiply-adds are written explicitly where wanted.
EXTRA ?=
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude -I$(CSRC) -Wall -Wno-unused-result $(EXTRA)
LIB := $(PKG)/libgnsship.so
OBJDIR := build/obj
PROF_OBJDIR := build/prof_obj

OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.cpp.o,$(CPP_SRCS))

all: $(LIB) oracle

# The acquisition FFTs are plain f32 VALU work: SLP packing into v_pk_add/mul_f32 buys no rate on
# gfx950 (a packed f32 op issues in 4 cycles, a scalar one in 2) and costs register-pair moves
# and VGPRs (C3 search kernel: 128 VGPRs + scratch packed, 84 unpacked).  Same IEEE ops either way.
$(OBJDIR)/acq_kernel.o $(PROF_OBJDIR)/acq_kernel.o: HIPFLAGS += -fno-slp-vectorize
# The tracking engine's serial accumulations (trk_fast.hip) likewise: a dependent packed add issues
# several times slower than single-rate adds.
$(OBJDIR)/trk_fast.o $(PROF_OBJDIR)/trk_fast.o: HIPFLAGS += -fno-slp-vectorize

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x c++ -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -s -C oracle all
	-@test -d /root/reference && $(MAKE) -s -C oracle ref || true

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean

# C++ mirror-class test (links the product library and, as the checker, the oracle source)
MIRROR_TEST := tests/cpp/mirror_test
$(MIRROR_TEST): tests/cpp/mirror_test.cpp include/gnsship_cpp.hpp include/gnsship.h oracle/gnss_oracle.c oracle/avx_port.c $(LIB)
	gcc -O2 -fPIC -ffp-contract=off -std=gnu11 -c oracle/gnss_oracle.c -o build/gnss_oracle_test.o
	gcc -O2 -fPIC -ffp-contract=off -std=gnu11 -c oracle/avx_port.c -o build/avx_port_test.o
	g++ -O2 -std=c++17 -Iinclude tests/cpp/mirror_test.cpp build/gnss_oracle_test.o build/avx_port_test.o -o $@ -L$(PKG) -lgnsship -Wl,-rpath,'$$ORIGIN/../../$(PKG)' -lpthread -lm
all: $(MIRROR_TEST)

# Profiling variant (workgroup phase timestamps in corr_batch_kernel; scripts/corr_wg_profile.py)
PROF_LIB := scripts/libgnsship_prof.so
PROF_OBJS := $(patsubst $(CSRC)/%.hip,$(PROF_OBJDIR)/%.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,$(PROF_OBJDIR)/%.cpp.o,$(CPP_SRCS))
$(PROF_OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(PROF_OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DGNSSHIP_CORR_PROFILE -c $< -o $@
$(PROF_OBJDIR)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(PROF_OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x c++ -c $< -o $@
$(PROF_LIB): $(PROF_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(PROF_OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
prof: $(PROF_LIB)
.PHONY: prof

# Standalone receiver core (the Channel role over the C ABI: include/gnsship_receiver.hpp)
RX_TOOL := tools/gnsship_rx
$(RX_TOOL): tools/gnsship_rx.cpp include/gnsship_receiver.hpp include/gnsship_cpp.hpp include/gnsship.h $(LIB)
	g++ -O2 -std=c++17 -Wall -Iinclude tools/gnsship_rx.cpp -o $@ -L$(PKG) -lgnsship -Wl,-rpath,'$$ORIGIN/../$(PKG)' -lpthread -lm
all: $(RX_TOOL)
