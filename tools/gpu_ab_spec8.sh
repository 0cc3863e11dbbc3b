#!/bin/bash
# The config-3 train kernel's GPU tests, then paired A/B of config 3 against
# build/prev.  Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec8.py tests/test_gpu_depth.py tests/test_gpu_range.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_spec8_tests.txt 2>&1 || { tail -20 gpurun_out/ab_spec8_tests.txt; exit 1; }
tail -2 gpurun_out/ab_spec8_tests.txt
CONFIG=3 NAMES=prev bash tools/ab_libs.sh || exit 1
