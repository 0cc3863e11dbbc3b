#!/bin/bash
# spec8 with the vector role on the older wave of each SIMD (variant vfirst):
# its tests, then paired A/B of config 3, three rounds.
set -o pipefail
mkdir -p gpurun_out
XH_LIB_PATH=build/vfirst/libxylo_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_spec8.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_vfirst_tests.txt 2>&1 || { tail -20 gpurun_out/ab_vfirst_tests.txt; exit 1; }
tail -2 gpurun_out/ab_vfirst_tests.txt
REPS=3 CONFIG=3 NAMES="vfirst" bash tools/ab_libs.sh || exit 1
