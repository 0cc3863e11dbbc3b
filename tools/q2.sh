#!/bin/bash
# Config 2 (32-bin 1-D [64,64]): the parity subset at that shape (goldens,
# oracle multi-group cases, kernel info), then bench A/B of the default train
# kernel against XH_TRAIN_KERNEL=f32 (diagnostic override).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/grad_units.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_boundary.py -k "b32d1 or 32-1 or kernel_info" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/q2_tests.txt 2>&1 || { tail -40 gpurun_out/q2_tests.txt; exit 1; }
tail -2 gpurun_out/q2_tests.txt
for rep in 1 2; do
for k in default f32; do
  if [ $k = default ]; then unset XH_TRAIN_KERNEL; A=""; else export XH_TRAIN_KERNEL=$k; A="--allow-kernel-override"; fi
  timeout -k 10 200 python -u bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline $A > gpurun_out/q2_bench_$k.json 2> gpurun_out/q2_bench_$k.err || { tail gpurun_out/q2_bench_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q2_bench_$k.json'));r=d['roofline'];print('$k', d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], r['peak'])"
done
done
