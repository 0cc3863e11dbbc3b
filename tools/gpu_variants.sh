#!/bin/bash
# Bench each variant library build/<v>/libxylo_hip.so (make variant) on one
# box, with the phase trace when the build has it.  VARS="t0 t1 ..."
set -o pipefail
mkdir -p gpurun_out
for v in ${VARS}; do
  XH_LIB_PATH=$PWD/build/$v/libxylo_hip.so XH_PHASE_TRACE=1 timeout -k 10 120 \
    python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/var_$v.log 2>&1 || { tail -5 gpurun_out/var_$v.log; exit 1; }
  echo "$v $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/var_$v.log) $(grep -o '"value": [0-9.]*' gpurun_out/var_$v.log | head -1)"
  grep -E "phase trace|kernel stamps|workgroup|placement|  cu " gpurun_out/var_$v.log | tail -11 | cut -c1-400
done
