#!/bin/bash
# Full GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel trace and
# the two HBM counter passes.  Every GPU step has its own time limit and the
# script stops at the first failure (no retries).
#   TAG=r01b bash tools/gpu_round.sh          (SKIP_TESTS=1 to bench/profile only)
set -o pipefail
TAG=${TAG:-rXX}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
PROF_ARGS="--steps 5 --warmup 1 --no-cpu-baseline"

if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider \
      --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; tail -2 $O/smoke.log
  [ $rc -ne 0 ] && exit $rc
fi

timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log | cut -c1-2000
[ $rc -ne 0 ] && exit $rc

rm -rf $O/prof_trace $O/prof_fetch $O/prof_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run \
    -- python3 bench.py $PROF_ARGS > $O/prof_trace.log 2>&1
rc=$?; tail -1 $O/prof_trace.log | cut -c1-600
[ $rc -ne 0 ] && exit $rc
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run \
    -- python3 bench.py $PROF_ARGS > $O/prof_fetch.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $O/prof_fetch.log; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run \
    -- python3 bench.py $PROF_ARGS > $O/prof_write.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $O/prof_write.log; exit $rc; }
PROFILE_OUT=$O/profiles python tools/pmc_summary.py $TAG $O/prof_trace $O/prof_fetch $O/prof_write \
    > $O/pmc_summary.log 2>&1
rc=$?; cat $O/pmc_summary.log | head -20
[ $rc -ne 0 ] && exit $rc
# bench again with this pass's HBM counters in profiles/ (roofline.traffic)
cp $O/profiles/${TAG}_pmc_summary.json profiles/ &&
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $O/bench_final.log 2>&1
rc=$?; tail -1 $O/bench_final.log | cut -c1-2000
exit $rc
