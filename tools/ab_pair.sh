#!/bin/bash
# A/B of two library builds on one box: bench each twice, alternating.
#   build/base/libxylo_hip.so = A (make a copy first), in-tree lib = B
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export XH_LIB_PATH=$PWD/build/base/libxylo_hip.so; else unset XH_LIB_PATH; fi
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$v$r.log 2>&1 || exit $?
    echo "$v$r $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/ab_$v$r.log) $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v$r.log | tr '\n' ' ')"
  done
done
