#!/bin/bash
# Config-5 train kernel: the 128-bin parity subset (goldens, oracle
# multi-group cases, full-size properties), then bench A/B of the default
# kernel against XH_TRAIN_KERNEL=${1:-split128} (diagnostic override).
set -o pipefail
K=${1:-split128}
mkdir -p gpurun_out
rm -f gpurun_out/grad_units.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -k "b128 or B128 or 128-3 or 128 or gpu_vs_oracle" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/q5_tests.txt 2>&1 || { tail -40 gpurun_out/q5_tests.txt; exit 1; }
tail -2 gpurun_out/q5_tests.txt
for rep in 1 2; do
for k in $K default; do
  if [ $k = default ]; then unset XH_TRAIN_KERNEL; A=""; else export XH_TRAIN_KERNEL=$k; A="--allow-kernel-override"; fi
  timeout -k 10 200 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline $A > gpurun_out/q5_bench_$k.json 2> gpurun_out/q5_bench_$k.err || { tail gpurun_out/q5_bench_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q5_bench_$k.json'));r=d['roofline'];print('$k', d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], r['peak'])"
done
done
