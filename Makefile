# Builds the MI355X-native library (gfx950 only) in-tree:
#   dependence_free_rl_amd/libxylo_hip.so   (C ABI: include/xylo_hip.h)
# and the test-only CPU oracle (oracle/liboracle.so, oracle/_ref/ when the
# reference tree is present).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := dependence_free_rl_amd
SRC      := $(PKG)/csrc
LIB      := $(PKG)/libxylo_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall \
            -Wno-unused-result -Iinclude -I$(SRC)
OBJS     := $(SRC)/policy_kernels.o $(SRC)/value_kernels.o \
            $(SRC)/env_kernels.o $(SRC)/xylo_hip.o
HDRS     := $(SRC)/xh_device.h $(SRC)/xh_kernels.h include/xylo_hip.h

.PHONY: all lib oracle clean
all: lib oracle

lib: $(LIB)

$(SRC)/%.o: $(SRC)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SRC)/xylo_hip.o: $(SRC)/xylo_hip.cpp $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -L/opt/rocm/lib -lrccl \
	    -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle port
	@if [ -d /root/reference ]; then $(MAKE) -C oracle ref; fi

clean:
	rm -f $(OBJS) $(LIB)
