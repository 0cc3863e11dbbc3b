#!/bin/bash
# Ad-hoc GPU check: wave-priority alternation in the 64-bin train kernel
# (per slot / per phase) against the product, config 3.
set -o pipefail
export TMPDIR=/tmp
CFG=3 ROUNDS=2 bash tools/ab_lib.sh build/v8wh_prio1/libxylo_hip.so build/v8wh_prio2/libxylo_hip.so || exit 1
