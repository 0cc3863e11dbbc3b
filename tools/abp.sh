#!/bin/bash
# A/B builds of one train-kernel source: each "name:FLAGS" argument compiles
# $AB_SRC (default: the product policy_split8wp_kernels.hip) with FLAGS into
# build/ab_<name>/libxylo_hip.so in place of $AB_OBJ (run here);
# `tools/abp.sh run KERNEL name...` benches them on the box with
# XH_TRAIN_KERNEL=KERNEL (diagnostic builds only, never the product path).
set -o pipefail
AB_OBJ=${AB_OBJ:-policy_split8wp_kernels}
AB_SRC=${AB_SRC:-dependence_free_rl_amd/csrc/$AB_OBJ.hip}
if [ "$1" = run ]; then
  K=$2; shift 2
  mkdir -p gpurun_out
  for rep in 1 2; do
    for n in "$@"; do
      XH_TRAIN_KERNEL=$K XH_LIB_PATH=build/ab_$n/libxylo_hip.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --allow-kernel-override $BENCH_ARGS > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -3 gpurun_out/ab_$n.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n', d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['value'])"
    done
  done
  exit 0
fi
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -Idependence_free_rl_amd/csrc -mllvm -amdgpu-mfma-vgpr-form"
OBJS=$(ls dependence_free_rl_amd/csrc/*.o | grep -v "/$AB_OBJ.o")
for spec in "$@"; do
  n=${spec%%:*}; f=${spec#*:}
  mkdir -p build/ab_$n
  /opt/rocm/bin/hipcc $HF $f -Rpass-analysis=kernel-resource-usage -c $AB_SRC -o build/ab_$n/k.o 2>&1 | grep -E "error|Spill: [1-9]" | sed "s/^/$n: /"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab_$n/libxylo_hip.so build/ab_$n/k.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
