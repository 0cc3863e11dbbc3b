#!/bin/bash
# env-only A/B: product (4 bins per lane) vs venv8 / venv16 variants, two sizes
for rep in 1 2; do for v in ${VARS:-product venv8 venv16}; do
  if [ $v = product ]; then lib=dependence_free_rl_amd/libxylo_hip.so; else lib=build/$v/libxylo_hip.so; fi
  for n in 32768 1048576; do
    XH_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --env-only --envs $n --steps 20 --warmup 2 > gpurun_out/envab_${v}_$n.log 2>&1 || { echo "$v $n failed"; tail -3 gpurun_out/envab_${v}_$n.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/envab_${v}_$n.log').read().strip().splitlines()[-1]); print('$v', $n, d['value'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])"
  done; done; done
