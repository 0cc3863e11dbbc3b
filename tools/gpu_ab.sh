#!/bin/bash
# GPU tests, then the bench with the default kernels and with each XH_ABLATE
# value in $ABL (diagnostic variants; numbers only).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_ab.log
tail -3 gpurun_out/pytest_ab.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab0.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_ab0.log').read().strip().splitlines()[-1]);print('default',d['value'],d['roofline']['avg_launch_ms'],d['phase_ms_per_step'])"
for m in $ABL; do
  XH_ABLATE=$m timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab$m.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bench_ab$m.log').read().strip().splitlines()[-1]);print('ablate',$m,d['value'],d['roofline']['avg_launch_ms'],d['phase_ms_per_step'])"
done
