#!/bin/bash
# rollout A/B: per config, per lib: rollout ms per iteration
set -o pipefail
for c in 3 5; do
for rep in 1 2; do
for n in base ${RAB_VARIANTS:-pk2 pk4}; do
  if [ $n = base ]; then L=""; else L="XH_LIB_PATH=build/ab_$n/libxylo_hip.so"; fi
  env $L timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r_$n.json 2> gpurun_out/r_$n.err || { tail -3 gpurun_out/r_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r_$n.json'));print('c$c', '$n', d['phase_ms_per_step']['rollout'], d['value'])"
done; done; done
