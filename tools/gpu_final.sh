#!/bin/bash
# A round's closing evidence after gpu_profile.sh: the bench lines (citing
# the TAG's PMC summaries by library hash), then the whole GPU suite.
set -o pipefail
TAG=${TAG:-rXX} bash tools/gpu_benches.sh || exit 1
TAG=${TAG:-rXX} bash tools/gpu_tests.sh || exit 1
