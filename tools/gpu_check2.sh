#!/bin/bash
# GPU-box check: parity tests, smoke, the headline bench and the other
# configurations' bench lines.  Every GPU step has its own time limit; a
# failure stops the script (no retries).
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-3000
for c in 2 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_c$c.log 2>&1 || { tail -5 $O/bench_c$c.log; exit 1; }
  tail -1 $O/bench_c$c.log | cut -c1-1500
done
exit $rc
