#!/bin/bash
# GPU tests of the 32-bin and 64-bin split train kernels (PPO and KL-PPO),
# then paired A/B against build/prev: config 2 (PPO) and config 3's shape
# under KL-PPO.  Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_klppo.py tests/test_gpu_parity.py tests/test_gpu_depth.py tests/test_gpu_range.py tests/test_gpu_spec8.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_mask_tests.txt 2>&1 || { tail -20 gpurun_out/ab_mask_tests.txt; exit 1; }
tail -2 gpurun_out/ab_mask_tests.txt
CONFIG=2 NAMES=prev bash tools/ab_libs.sh || exit 1
CONFIG=3 EXTRA="--algo klppo" NAMES=prev bash tools/ab_libs.sh || exit 1
