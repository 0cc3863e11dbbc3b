#!/bin/bash
# spec8 iteration: its GPU tests, then the ablation timings (tools/ab_spec8.sh)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05c}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_spec8.py > gpurun_out/${TAG}_spec8_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_spec8_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_spec8_tests.txt
bash tools/ab_spec8.sh
