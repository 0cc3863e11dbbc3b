#!/bin/bash
# Ad-hoc GPU check: KL-PPO on the split kernel (and the f32 reference), the
# config-3 A/B (PPO kernel unchanged), the KL-PPO side line.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
rm -f $O/grad_units.jsonl
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_klppo.py > $O/chk_kl.txt 2>&1 || { tail -40 $O/chk_kl.txt; exit 1; }
grep -E "PASS|FAIL" $O/chk_kl.txt | tail -5
CFG=3 ROUNDS=2 bash tools/ab_lib.sh build/base/libxylo_hip.so || exit 1
timeout -k 10 300 python -u bench.py --algo klppo --no-cpu-baseline > $O/chk_kl_bench.json 2> $O/chk_kl_bench.err || { tail -5 $O/chk_kl_bench.err; exit 1; }
tail -1 $O/chk_kl_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('KL', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline'].get('kernel'), d.get('phase_ms_per_step'))"
