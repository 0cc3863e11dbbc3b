#!/bin/bash
# Ad-hoc GPU check: the 128-bin KL build with LDS-direct q staging -- its
# oracle tests and KL-PPO at config 5's shape.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_klppo.py -k "b128 or recorded" > $O/chk_kl.txt 2>&1 || { tail -40 $O/chk_kl.txt; exit 1; }
tail -1 $O/chk_kl.txt
for r in 1 2; do
timeout -k 10 300 python -u bench.py --config 5 --algo klppo --no-cpu-baseline > $O/kl5.json 2> $O/kl5.err || { tail -5 $O/kl5.err; exit 1; }
tail -1 $O/kl5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('KL c5', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'])"
done
