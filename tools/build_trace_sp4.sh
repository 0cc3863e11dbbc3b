#!/bin/bash
# Diagnostic phase-stamp build of the wave-specialised config-2 train kernel
# (build/tsp4/; loaded through XH_LIB_PATH with XH_PHASE_TRACE=1 -- and
# XH_PHASE_TRACE_WAVES=1 for per-wave means -- never by the product path).
# Slots per group: A work, A barrier, B work, B barrier (xylo_hip.cpp prints
# them under the 8-wave kernel's labels: fwd = A work, bar1 = A barrier,
# softmax = B work, layer3 = B barrier).  $1: extra kernel flags.
set -e
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -Idependence_free_rl_amd/csrc"
D=build/tsp4${2:+_$2}
mkdir -p $D
/opt/rocm/bin/hipcc $HF -DXH_DIAG_TRACE=1 -c dependence_free_rl_amd/csrc/policy_kernels.hip -o $D/policy_kernels.o
/opt/rocm/bin/hipcc $HF -DXH_DIAG_TRACE=1 -c dependence_free_rl_amd/csrc/xylo_hip.cpp -o $D/xylo_hip.o
/opt/rocm/bin/hipcc $HF -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize -DXH_DIAG_TRACE=1 $1 -c dependence_free_rl_amd/csrc/policy_spec4_kernels.hip -o $D/policy_spec4_kernels.o
OBJS=$(ls dependence_free_rl_amd/csrc/*.o | grep -v "/policy_kernels.o\|/policy_spec4_kernels.o\|/xylo_hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libxylo_hip.so $D/policy_kernels.o $D/xylo_hip.o $D/policy_spec4_kernels.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
