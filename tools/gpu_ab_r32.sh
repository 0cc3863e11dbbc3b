#!/bin/bash
# The 32-bin split rollout at one env per wave: the tests that run it
# (full-size split vs f32 rollout, parity goldens, KL-PPO, boundaries), then
# paired A/B of config 2 against the two-env build (variant r32two).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_klppo.py tests/test_gpu_boundary.py tests/test_gpu_model_api.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_r32_tests.txt 2>&1 || { tail -25 gpurun_out/ab_r32_tests.txt; exit 1; }
tail -2 gpurun_out/ab_r32_tests.txt
REPS=3 CONFIG=2 NAMES="r32two" bash tools/ab_libs.sh || exit 1
