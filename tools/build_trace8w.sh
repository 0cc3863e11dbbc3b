#!/bin/bash
# Diagnostic phase-stamp build of the 8-wave train kernel (build/t8/; loaded
# through XH_LIB_PATH with XH_PHASE_TRACE=1, never by the product path).
set -e
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -Idependence_free_rl_amd/csrc"
mkdir -p build/t8
/opt/rocm/bin/hipcc $HF -DXH_DIAG_TRACE=1 -c dependence_free_rl_amd/csrc/policy_kernels.hip -o build/t8/policy_kernels.o
/opt/rocm/bin/hipcc $HF -mllvm -amdgpu-mfma-vgpr-form -DXH_DIAG_TRACE=1 -c dependence_free_rl_amd/csrc/policy_split8w_kernels.hip -o build/t8/policy_split8w_kernels.o
OBJS=$(ls dependence_free_rl_amd/csrc/*.o | grep -v "/policy_kernels.o\|/policy_split8w_kernels.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/t8/libxylo_hip.so build/t8/policy_kernels.o build/t8/policy_split8w_kernels.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
