#!/bin/bash
# The config-3 train kernel's tests on the W2-lo-in-LDS variant, then paired
# A/B of config 3 (product, wlo), three rounds.  Each step has its own limit.
set -o pipefail
mkdir -p gpurun_out
XH_LIB_PATH=build/wlo/libxylo_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_spec8.py tests/test_gpu_range.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_wlo_tests.txt 2>&1 || { tail -20 gpurun_out/ab_wlo_tests.txt; exit 1; }
tail -2 gpurun_out/ab_wlo_tests.txt
REPS=3 CONFIG=3 NAMES="wlo" bash tools/ab_libs.sh || exit 1
