#!/bin/bash
# Ad-hoc GPU check of the current change (tests named by -k, parity, bench lines)
set -o pipefail
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_boundary.py tests/test_gpu_scale.py -k "wide_slot0 or kernel_info or split_rollout or other_configs or gpu_vs_oracle" > $O/r04d_tests.txt 2>&1 || { tail -30 $O/r04d_tests.txt; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "b32 or b64" > $O/r04d_parity.txt 2>&1 || { tail -30 $O/r04d_parity.txt; exit 1; }
for c in 2 3 5; do timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/r04d_b$c.log 2>&1 || { tail -5 $O/r04d_b$c.log; exit 1; }; done
tail -3 $O/r04d_tests.txt; tail -2 $O/r04d_parity.txt
for c in 2 3 5; do tail -1 $O/r04d_b$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:30], d['ms_per_step'], d['phase_ms_per_step'])"; done
