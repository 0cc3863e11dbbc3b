#!/bin/bash
# Config-2 probe: train-epoch time against the groups per workgroup (envs
# 2048 .. 16384 = J 8 .. 64), then a kernel trace of the iteration (the gaps
# between launches).
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
for n in 2048 4096 8192 16384; do
  timeout -k 10 200 python -u bench.py --config 2 --envs $n --no-cpu-baseline > $O/c2p_$n.log 2>&1 || { tail -5 $O/c2p_$n.log; exit 1; }
  tail -1 $O/c2p_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], d['phase_ms_per_step'])"
done
rm -rf $O/c2trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2trace -o run \
    -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/c2trace.log 2>&1 || { tail -5 $O/c2trace.log; exit 1; }
find $O/c2trace -name "*kernel_trace.csv" | head -2
