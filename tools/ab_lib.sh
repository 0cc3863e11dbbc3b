#!/bin/bash
# Paired A/B of the bench between the product library and variant libraries
# on one box: rounds x (product, each XH_LIB_PATH variant), config $CFG.
#   bash tools/ab_lib.sh build/dw2bf16/libxylo_hip.so [more libs]
set -o pipefail
O=gpurun_out
CFG=${CFG:-3}
ROUNDS=${ROUNDS:-2}
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for lib in product "$@"; do
    tag=$(echo $lib | tr '/.' '__')
    if [ $lib = product ]; then unset XH_LIB_PATH; else export XH_LIB_PATH=$lib; fi
    timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline > $O/ab_${tag}_$r.json 2> $O/ab_${tag}_$r.err || { tail -5 $O/ab_${tag}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/ab_${tag}_$r.json').read().strip().splitlines()[-1])
r=d['roofline']; print('%-40s r$r value %.4gM ms/it %.3f train %.4f ms frac %.3f peak %s' % ('$lib', d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['peak']))"
  done
done
