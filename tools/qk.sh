#!/bin/bash
# A train kernel under XH_TRAIN_KERNEL=$1: the config-3 parity subset
# (goldens at the 64-bin shape, oracle multi-group cases), then bench A/B
# against the default kernel (diagnostic override, never the product path).
set -o pipefail
K=$1
mkdir -p gpurun_out
rm -f gpurun_out/grad_units.jsonl
XH_TRAIN_KERNEL=$K timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -k "b64d2 or B64 or ppo-64 or gpu_vs_oracle" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/qk_tests.txt 2>&1 || { tail -40 gpurun_out/qk_tests.txt; exit 1; }
tail -2 gpurun_out/qk_tests.txt
for rep in 1 2; do
for k in $K default; do
  if [ $k = default ]; then unset XH_TRAIN_KERNEL; A=""; else export XH_TRAIN_KERNEL=$k; A="--allow-kernel-override"; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $A > gpurun_out/qk_bench_$k.json 2> gpurun_out/qk_bench_$k.err || { tail gpurun_out/qk_bench_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/qk_bench_$k.json'));r=d['roofline'];print('$k', d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], r['peak'])"
done
done
