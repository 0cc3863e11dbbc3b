#!/bin/bash
# The whole GPU test suite in one process (the driver's round-end tier), its
# log and the per-case gradient-error log copied for profiles/.
set -o pipefail
O=gpurun_out
TAG=${TAG:-rXX}
mkdir -p $O/profiles
rm -f $O/grad_units.jsonl $O/sampling_agreement.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/profiles/${TAG}_gpu_tests.txt 2>&1
rc=$?
tail -5 $O/profiles/${TAG}_gpu_tests.txt
[ -f $O/grad_units.jsonl ] && cp $O/grad_units.jsonl $O/profiles/${TAG}_grad_units.jsonl
[ -f $O/sampling_agreement.jsonl ] && cp $O/sampling_agreement.jsonl $O/profiles/${TAG}_sampling_agreement.jsonl
exit $rc
