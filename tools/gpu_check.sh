#!/bin/bash
# Ad-hoc GPU check: paired A/B benches of the product against variant libs.
set -o pipefail
export TMPDIR=/tmp
CFG=3 ROUNDS=3 bash tools/ab_lib.sh build/base/libxylo_hip.so build/v8wh_pt0/libxylo_hip.so build/v8wh_dw0/libxylo_hip.so build/v8wh_pt0dw0/libxylo_hip.so
