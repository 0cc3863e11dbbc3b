#!/bin/bash
# Ad-hoc GPU check: recorded distributions on the split rollouts.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_klppo.py -k recorded > $O/chk_rec.txt 2>&1 || { tail -40 $O/chk_rec.txt; exit 1; }
grep -E "PASS|FAIL" $O/chk_rec.txt | tail -4
