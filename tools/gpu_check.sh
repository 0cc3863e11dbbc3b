#!/bin/bash
# Ad-hoc GPU check: config-3 parity subset, then the paired A/B product vs
# build/old8 (the config-3 train kernel before the prologue rework).
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_depth.py tests/test_gpu_range.py -k "b64 or 64-2 or c3" > $O/chk_tests.txt 2>&1 || { tail -30 $O/chk_tests.txt; exit 1; }
tail -2 $O/chk_tests.txt
CFG=3 ROUNDS=3 bash tools/ab_lib.sh build/old8/libxylo_hip.so
