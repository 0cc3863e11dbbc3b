#!/bin/bash
# The config-3 train kernel's GPU tests on the MK16 variant (as the product
# library through XH_LIB_PATH), then paired A/B of config 3: product, prev,
# mk16, three rounds.  Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
XH_LIB_PATH=build/mk16/libxylo_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_spec8.py tests/test_gpu_depth.py tests/test_gpu_range.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_mk16_tests.txt 2>&1 || { tail -20 gpurun_out/ab_mk16_tests.txt; exit 1; }
tail -2 gpurun_out/ab_mk16_tests.txt
REPS=3 CONFIG=3 NAMES="prev mk16" bash tools/ab_libs.sh || exit 1
