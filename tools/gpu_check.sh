#!/bin/bash
# Ad-hoc GPU check: the KL-PPO builds (64 / 128 / 32 bins) against the
# oracle; config 2 A/B (its PPO kernel unchanged); KL-PPO at config 2's shape.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
rm -f $O/grad_units.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_klppo.py > $O/chk_kl.txt 2>&1 || { tail -40 $O/chk_kl.txt; exit 1; }
grep -E "PASS|FAIL" $O/chk_kl.txt | tail -12
CFG=2 ROUNDS=2 bash tools/ab_lib.sh build/base/libxylo_hip.so || exit 1
timeout -k 10 300 python -u bench.py --config 2 --algo klppo --no-cpu-baseline > $O/kl2.json 2> $O/kl2.err || { tail -5 $O/kl2.err; exit 1; }
tail -1 $O/kl2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('KL c2', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], r['rows_per_launch'])"
XH_TRAIN_KERNEL=f32 timeout -k 10 300 python -u bench.py --config 2 --algo klppo --no-cpu-baseline --allow-kernel-override > $O/kl2f.json 2> $O/kl2f.err || { tail -5 $O/kl2f.err; exit 1; }
tail -1 $O/kl2f.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('KL c2 f32', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'])"
