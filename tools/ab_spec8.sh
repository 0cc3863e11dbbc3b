#!/bin/bash
# Ablation timing of the wave-specialised train kernel: the config-3 bench's
# policy-train launch time with the product library and with the
# XH_SP8_ABLATE variant libraries (build/abl<bits>/, `make variant
# V=abl<bits> VSRC=policy_spec8_kernels VFLAGS=-DXH_SP8_ABLATE=<bits>`;
# wrong results by design, timings only).
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r05c}_ab_spec8.txt
: > $OUT
for v in product ${VARIANTS:-1 2 4 8 16 32}; do
  if [ $v = product ]; then lib=dependence_free_rl_amd/libxylo_hip.so; else lib=build/abl$v/libxylo_hip.so; fi
  XH_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "
import json,sys
d=json.load(open('gpurun_out/ab_$v.json'))
print('$v', d['roofline']['kernel'], 'train ms', d['roofline']['avg_launch_ms'], 'value', d['value'])" | tee -a $OUT
done
