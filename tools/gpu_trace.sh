set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_venv.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/venv.log 2>&1; tail -3 gpurun_out/venv.log
XH_LIB_PATH=$PWD/build/diag/libxylo_hip.so XH_PHASE_TRACE=1 timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/trace_c3.log 2>&1 || { tail -5 gpurun_out/trace_c3.log; exit 1; }
grep "phase trace" gpurun_out/trace_c3.log | tail -3
timeout -k 10 300 python -u bench.py --rollout-steps 32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_T32.log 2>&1 || { tail -5 gpurun_out/bench_T32.log; exit 1; }
tail -1 gpurun_out/bench_T32.log | cut -c1-600
