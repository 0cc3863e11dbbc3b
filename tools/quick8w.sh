set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/grad_units.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -k "b64d2 or B64 or ppo-64 or split_train or c3_full or gpu_vs_oracle" -v --timeout 200 --timeout-method thread -p no:cacheprovider -x > gpurun_out/q8w_tests.txt 2>&1 || { tail -30 gpurun_out/q8w_tests.txt; exit 1; }
tail -3 gpurun_out/q8w_tests.txt
for k in split4w default; do
  if [ $k = default ]; then unset XH_TRAIN_KERNEL; A=""; else export XH_TRAIN_KERNEL=$k; A="--allow-kernel-override"; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $A > gpurun_out/q8w_bench_$k.json 2> gpurun_out/q8w_bench_$k.err || { cat gpurun_out/q8w_bench_$k.err | tail; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q8w_bench_$k.json'));print('$k', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['phase_ms_per_step'])"
done
XH_LIB_PATH=build/t8/libxylo_hip.so XH_PHASE_TRACE=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/t8.json 2> gpurun_out/t8.err || { tail -5 gpurun_out/t8.err; exit 1; }
grep "phase trace" gpurun_out/t8.err | tail -1
