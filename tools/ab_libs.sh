#!/bin/bash
# Config-3 train-kernel time of the product library and of variant
# libraries build/<name>/libxylo_hip.so (timings only), in the order given,
# twice (alternating) to expose drift.  EXTRA: more bench.py arguments
# (e.g. "--algo klppo").
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for v in product $NAMES; do
  if [ $v = product ]; then lib=dependence_free_rl_amd/libxylo_hip.so; else lib=build/$v/libxylo_hip.so; fi
  XH_LIB_PATH=$lib timeout -k 10 200 python bench.py --config ${CONFIG:-3} --steps 5 --warmup 2 --no-cpu-baseline $EXTRA \
    > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err || { echo "$v failed"; tail -5 gpurun_out/abl_$v.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/abl_$v.json'))
ph=d.get('phase_ms_per_step',{})
print('$v', 'train ms', d['roofline']['avg_launch_ms'], 'value', d['value'], 'phases', {k: v for k, v in ph.items() if k != 'source'})"
done
done
