#!/bin/bash
# The 128-bin rollout's half-unit split: the tests that run it (full-size
# split vs f32 rollout, parity and KL-PPO at 128 bins, the config-5 global
# workload, boundaries), then paired A/B of config 5 against build/prev.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_klppo.py tests/test_gpu_global.py tests/test_gpu_boundary.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_r128h_tests.txt 2>&1 || { tail -25 gpurun_out/ab_r128h_tests.txt; exit 1; }
tail -2 gpurun_out/ab_r128h_tests.txt
REPS=3 CONFIG=5 NAMES="prev" bash tools/ab_libs.sh || exit 1
