#!/bin/bash
# Ad-hoc GPU check of the current change: the named tests, then bench lines.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./build/probe_graph > $O/probe_graph.txt 2>&1 || { cat $O/probe_graph.txt; exit 1; }
cat $O/probe_graph.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_depth.py tests/test_gpu_range.py tests/test_gpu_boundary.py tests/test_gpu_shards.py -k "b32 or 32-1 or c2 or b128 or 128-3 or b64 or 64-2 or wide or split_rollout or wave_rollout or shard or env_state or override" > $O/chk_tests.txt 2>&1 || { tail -30 $O/chk_tests.txt; exit 1; }
tail -2 $O/chk_tests.txt
for c in 2 5; do timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/chk_b$c.log 2>&1 || { tail -5 $O/chk_b$c.log; exit 1; }
  tail -1 $O/chk_b$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:18], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['iteration_roofline']['frac'], d['phase_ms_per_step'])"; done
XH_LIB_PATH=build/t4h/libxylo_hip.so XH_PHASE_TRACE=1 timeout -k 10 200 python -u bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/t4h.log 2> $O/t4h.err || { tail -5 $O/t4h.err; exit 1; }
grep -m 2 "phase trace\|kernel stamps" $O/t4h.err
CFG=3 ROUNDS=2 bash tools/ab_lib.sh build/p8/libxylo_hip.so
timeout -k 10 300 python -u bench.py --config 3 --algo klppo --no-cpu-baseline > $O/chk_kl.log 2>&1 || { tail -5 $O/chk_kl.log; exit 1; }
tail -1 $O/chk_kl.log | cut -c1-600
CFG=5 ROUNDS=2 bash tools/ab_lib.sh build/nofold/libxylo_hip.so
