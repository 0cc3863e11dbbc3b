#!/bin/bash
# GPU-box check: parity tests then the 1-GPU bench.  Every GPU step has its
# own time limit; a crash / fault / timeout stops the script (no retries).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
tail -2 gpurun_out/bench.log | cut -c1-1500
exit $rc
