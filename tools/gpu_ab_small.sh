#!/bin/bash
# Config 2's small kernels: the value tests (fused W0 prep bit-identical to the
# separate item kernel), then paired A/B at config 2 of the W0 fusion (an
# environment switch) and of variant libraries (slab reduce split, value
# forward grid).  Each GPU step has its own limit.
set -o pipefail
TESTS=tests/test_gpu_value.py CONFIG=2 ENVA="XH_W0_FUSE=0" ENVB="XH_W0_FUSE=1" REPS=3 EXTRA=--allow-kernel-override bash tools/gpu_ab_env.sh || exit 1
REPS=2 CONFIG=2 NAMES="slab16 slab32 vgrid2" bash tools/ab_libs.sh || exit 1
REPS=1 CONFIG=3 NAMES="slab16 vgrid2" bash tools/ab_libs.sh || exit 1
