#!/bin/bash
# A/B variants of the 8-wave train kernel: each argument "name:FLAGS" builds
# build/ab_<name>/libxylo_hip.so with policy_split8w_kernels.hip compiled
# with FLAGS (run here); `tools/ab8w.sh run name...` benches them on the box
# (XH_LIB_PATH; diagnostic builds only, never the product path).
set -o pipefail
if [ "$1" = run ]; then
  shift
  mkdir -p gpurun_out
  for rep in 1 2; do
    for n in "$@"; do
      XH_LIB_PATH=build/ab_$n/libxylo_hip.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -3 gpurun_out/ab_$n.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['value'])"
    done
  done
  exit 0
fi
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -Idependence_free_rl_amd/csrc -mllvm -amdgpu-mfma-vgpr-form"
OBJS=$(ls dependence_free_rl_amd/csrc/*.o | grep -v "/policy_split8w_kernels.o")
for spec in "$@"; do
  n=${spec%%:*}; f=${spec#*:}
  mkdir -p build/ab_$n
  /opt/rocm/bin/hipcc $HF $f -Rpass-analysis=kernel-resource-usage -c dependence_free_rl_amd/csrc/policy_split8w_kernels.hip -o build/ab_$n/k.o 2>&1 | grep -E "error|Spill: [1-9]" | sed "s/^/$n: /"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab_$n/libxylo_hip.so build/ab_$n/k.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
