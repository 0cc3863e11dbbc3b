#!/bin/bash
# Config 3 (the headline 64-bin shape): the parity subset on the product
# library, then `tools/abp.sh run` over the A/B builds named as arguments.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/grad_units.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -k "b64d2 or B64 or ppo-64 or gpu_vs_oracle or split_train" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/q3_tests.txt 2>&1 || { tail -40 gpurun_out/q3_tests.txt; exit 1; }
tail -2 gpurun_out/q3_tests.txt
[ $# -gt 0 ] && bash tools/abp.sh run "" "$@"
exit 0
