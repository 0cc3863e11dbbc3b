#!/bin/bash
# VGPR / scratch / occupancy of the kernels whose mangled name matches $1
# (default: the policy train kernels), from the compiler's resource remarks.
pat=${1:-policy_train}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude \
  -Idependence_free_rl_amd/csrc -Rpass-analysis=kernel-resource-usage \
  -c ${2:-dependence_free_rl_amd/csrc/policy_kernels.hip} -o /tmp/regs.o 2>&1 |
  grep -A9 -E "Function Name: .*${pat}" |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" |
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//'
