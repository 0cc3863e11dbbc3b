#!/bin/bash
# Round-5 check of the wave-specialised config-3 train kernel: its parity
# tests (against the oracle and split8wh), the depth / wide-range tests at
# the config-3 shape, then paired bench lines (spec8 default, split8wh).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05c}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_spec8.py tests/test_gpu_depth.py tests/test_gpu_range.py \
  > gpurun_out/${TAG}_spec8_tests.txt 2>&1 || { tail -40 gpurun_out/${TAG}_spec8_tests.txt; exit 1; }
tail -5 gpurun_out/${TAG}_spec8_tests.txt
for k in default split8wh default split8wh; do
  if [ $k = default ]; then
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/${TAG}_ab_bench.jsonl || exit 1
  else
    XH_TRAIN_KERNEL=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/${TAG}_ab_bench.jsonl || exit 1
  fi
  tail -1 gpurun_out/${TAG}_ab_bench.jsonl | cut -c1-400
done
