#!/bin/bash
# Ad-hoc GPU check: the Dense GEMMs' LDS padding (4 = product, 1, 2) --
# value-net bit-identity on a variant, A/B at configs 5 and 3.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
XH_LIB_PATH=build/vpad2/libxylo_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_value.py > $O/chk_pad.txt 2>&1 || { tail -30 $O/chk_pad.txt; exit 1; }
tail -1 $O/chk_pad.txt
for c in 5 3; do CFG=$c ROUNDS=2 bash tools/ab_lib.sh build/vpad1/libxylo_hip.so build/vpad2/libxylo_hip.so || exit 1; done
