#!/bin/bash
# policy_train ablation sweep (diagnostics; outputs are wrong by design)
mkdir -p gpurun_out
for m in ${ABL:-0 1 2 3 4 8 7 15}; do
  XH_ABLATE=$m timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$m.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/abl_$m.log').read().strip().splitlines()[-1]);print('ablate',$m,d['roofline']['avg_launch_ms'])"
done
