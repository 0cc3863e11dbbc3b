#!/bin/bash
# Paired A/B of one library under an environment switch: bench.py --config
# $CONFIG with "$ENVA" and with "$ENVB" (e.g. ENVA="XH_W0_FUSE=0" ENVB=""),
# alternating, REPS rounds; optional pytest files first (TESTS).  Each GPU
# step has its own limit.  Kernel-selection switches need
# EXTRA=--allow-kernel-override (bench.py refuses them otherwise).
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_env_tests.txt 2>&1 || { tail -20 gpurun_out/ab_env_tests.txt; exit 1; }
  tail -2 gpurun_out/ab_env_tests.txt
fi
for rep in $(seq ${REPS:-3}); do
  for side in A B; do
    if [ $side = A ]; then e="$ENVA"; else e="$ENVB"; fi
    env $e timeout -k 10 200 python bench.py --config ${CONFIG:-3} --steps 5 --warmup 2 --no-cpu-baseline $EXTRA \
      > gpurun_out/abe_$side.json 2> gpurun_out/abe_$side.err || { echo "$side failed"; tail -5 gpurun_out/abe_$side.err; exit 1; }
    python -c "
import json
d=json.load(open('gpurun_out/abe_$side.json'))
ph=d.get('phase_ms_per_step',{})
print('$side [$e]', 'ms/step', d['ms_per_step'], 'value', round(d['value']), 'phases', {k: v for k, v in ph.items() if k != 'source'})"
  done
done
