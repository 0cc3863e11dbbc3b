#!/bin/bash
# policy_train phase-ablation sweep on the diagnostic library (make diag;
# outputs are wrong by design, timings only).  Bits of XH_ABLATE in the 8-wave
# kernel: 4 = no layer-2 forward MFMAs, 8 = trivial loss gradient (no
# softmax / clipped surrogate), 16 = no dH1 MFMAs, 32 = no dW2 MFMAs (nor the
# dW1 VALU work riding in them).
mkdir -p gpurun_out
export XH_LIB_PATH=$PWD/build/diag/libxylo_hip.so
for m in ${ABL:-0 4 8 16 32 48 60}; do
  XH_ABLATE=$m timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$m.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/abl_$m.log').read().strip().splitlines()[-1]);print('ablate',$m,d['roofline']['avg_launch_ms'],d['phase_ms_per_step'])"
done
