export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_team.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_team.log
tail -4 gpurun_out/pytest_team.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_team.log 2>&1 || exit $?
tail -1 gpurun_out/bench_team.log
XH_TRAIN_KERNEL=8 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_t8.log 2>&1 || exit $?
tail -1 gpurun_out/bench_t8.log
