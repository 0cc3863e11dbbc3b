#!/bin/bash
# The 128-bin split rollout at 8 waves per workgroup (variant r128w8): its
# full-size rollout test, then paired A/B of config 5 against the product.
set -o pipefail
mkdir -p gpurun_out
XH_LIB_PATH=build/r128w8/libxylo_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -k "split_rollout and ac" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_r128_tests.txt 2>&1 || { tail -20 gpurun_out/ab_r128_tests.txt; exit 1; }
tail -2 gpurun_out/ab_r128_tests.txt
REPS=3 CONFIG=5 NAMES="r128w8" bash tools/ab_libs.sh || exit 1
