#!/bin/bash
# Pipelined 4-wave train kernel: config-3 parity subset (the default kernel),
# then bench A/B against the pipelined 8-wave one (XH_TRAIN_KERNEL=split8wp).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/grad_units.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py tests/test_gpu_boundary.py -k "b64d2 or B64 or ppo-64 or gpu_vs_oracle or shard or kernel" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/q4p_tests.txt 2>&1 || { tail -40 gpurun_out/q4p_tests.txt; exit 1; }
tail -3 gpurun_out/q4p_tests.txt
for rep in 1 2; do
for k in split8wp default; do
  if [ $k = default ]; then unset XH_TRAIN_KERNEL; A=""; else export XH_TRAIN_KERNEL=$k; A="--allow-kernel-override"; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $A > gpurun_out/q4p_bench_$k.json 2> gpurun_out/q4p_bench_$k.err || { tail gpurun_out/q4p_bench_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q4p_bench_$k.json'));print('$k', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
done
