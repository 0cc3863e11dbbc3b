#!/bin/bash
# Diagnostic phase-stamp build of the pipelined config-2 (4-wave) f16-pair train kernel (build/t4h/;
# loaded through XH_LIB_PATH with XH_PHASE_TRACE=1 -- XH_PHASE_TRACE_WAVES=1
# adds per-wave means -- never by the product path).  $1: extra flags for the
# kernel file (A/B of a trace build).
set -e
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -Idependence_free_rl_amd/csrc"
D=build/t4h${2:+_$2}
mkdir -p $D
/opt/rocm/bin/hipcc $HF -DXH_DIAG_TRACE=1 -c dependence_free_rl_amd/csrc/policy_kernels.hip -o $D/policy_kernels.o
/opt/rocm/bin/hipcc $HF -DXH_DIAG_TRACE=1 -c dependence_free_rl_amd/csrc/xylo_hip.cpp -o $D/xylo_hip.o
/opt/rocm/bin/hipcc $HF -mllvm -amdgpu-mfma-vgpr-form -DXH_DIAG_TRACE=1 $1 -c dependence_free_rl_amd/csrc/policy_split4h_kernels.hip -o $D/policy_split4h_kernels.o
OBJS=$(ls dependence_free_rl_amd/csrc/*.o | grep -v "/policy_kernels.o\|/policy_split4h_kernels.o\|/xylo_hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libxylo_hip.so $D/policy_kernels.o $D/xylo_hip.o $D/policy_split4h_kernels.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
