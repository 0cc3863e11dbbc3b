#!/bin/bash
# Ad-hoc GPU check: the 64-bin KL build with LDS-direct q staging -- its
# oracle tests and the KL side line.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_klppo.py -k "b64" > $O/chk_kl.txt 2>&1 || { tail -40 $O/chk_kl.txt; exit 1; }
tail -1 $O/chk_kl.txt
for r in 1 2; do
timeout -k 10 300 python -u bench.py --algo klppo --no-cpu-baseline > $O/kl3.json 2> $O/kl3.err || { tail -5 $O/kl3.err; exit 1; }
tail -1 $O/kl3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('KL c3', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'])"
done
