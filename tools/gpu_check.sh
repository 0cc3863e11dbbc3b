#!/bin/bash
# Ad-hoc GPU check: the value step's split cap (256 = product, 512, 1024) at
# configs 2 and 3.
set -o pipefail
export TMPDIR=/tmp
CFG=2 ROUNDS=2 bash tools/ab_lib.sh build/vm512/libxylo_hip.so build/vm1024/libxylo_hip.so || exit 1
CFG=3 ROUNDS=2 bash tools/ab_lib.sh build/vm512/libxylo_hip.so build/vm1024/libxylo_hip.so || exit 1
