#!/bin/bash
# Ad-hoc GPU check: the PPO build's staging by LDS-direct loads (variant),
# parity on the variant, A/B at config 3.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
XH_LIB_PATH=build/v8wh_dma/libxylo_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "b64" > $O/chk_dma.txt 2>&1 || { tail -30 $O/chk_dma.txt; exit 1; }
tail -1 $O/chk_dma.txt
CFG=3 ROUNDS=2 bash tools/ab_lib.sh build/v8wh_dma/libxylo_hip.so || exit 1
