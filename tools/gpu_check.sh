#!/bin/bash
# Ad-hoc GPU check: the sharded tests (config-5 shape added) and the end list.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
rm -f $O/shard_sums.jsonl
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shards.py tests/test_gpu_parity.py -k "shard or learn_matches or klppo" > $O/chk_tests.txt 2>&1 || { tail -30 $O/chk_tests.txt; cat $O/shard_sums.jsonl; exit 1; }
tail -3 $O/chk_tests.txt; cat $O/shard_sums.jsonl
timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline > $O/chk_b3.log 2>&1 || { tail -5 $O/chk_b3.log; exit 1; }
tail -1 $O/chk_b3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['phase_ms_per_step'])"
