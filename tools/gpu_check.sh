#!/bin/bash
# Ad-hoc GPU check: the KL-PPO builds of the 64- and 128-bin train kernels
# against the oracle; config 5 A/B (its AC kernel unchanged); the KL side
# line at config 5's shape.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
rm -f $O/grad_units.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_klppo.py > $O/chk_kl.txt 2>&1 || { tail -40 $O/chk_kl.txt; exit 1; }
grep -E "PASS|FAIL" $O/chk_kl.txt | tail -6
CFG=5 ROUNDS=2 bash tools/ab_lib.sh build/base/libxylo_hip.so || exit 1
timeout -k 10 300 python -u bench.py --config 5 --algo klppo --no-cpu-baseline > $O/kl5.json 2> $O/kl5.err || { tail -5 $O/kl5.err; exit 1; }
tail -1 $O/kl5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('KL c5', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], r['rows_per_launch'])"
