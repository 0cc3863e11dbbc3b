#!/bin/bash
# GPU tests on the in-tree library, then an alternating A/B of variant
# libraries: VARS="base prod" (build/<v>/libxylo_hip.so), twice each.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for v in ${VARS}; do
    XH_LIB_PATH=$PWD/build/$v/libxylo_hip.so timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$v$r.log 2>&1 || { tail -5 gpurun_out/ab_$v$r.log; exit 1; }
    echo "$v$r $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/ab_$v$r.log) $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v$r.log | head -1) $(grep -o '"rollout": [0-9.]*' gpurun_out/ab_$v$r.log)"
  done
done
