#!/bin/bash
# Ad-hoc GPU check of the current change: the named tests, then bench lines.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_value.py tests/test_gpu_parity.py tests/test_gpu_scale.py -k "value or learn_matches or klppo or bench_json" > $O/chk_tests.txt 2>&1 || { tail -30 $O/chk_tests.txt; exit 1; }
tail -3 $O/chk_tests.txt
for c in 2 3 5; do timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/chk_b$c.log 2>&1 || { tail -5 $O/chk_b$c.log; exit 1; }
  tail -1 $O/chk_b$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:18], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['iteration_roofline']['frac'], d['phase_ms_per_step'])"; done
rm -rf $O/c2trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2trace -o run \
    -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/c2trace.log 2>&1 || { tail -5 $O/c2trace.log; exit 1; }
