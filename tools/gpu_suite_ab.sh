#!/bin/bash
# The whole GPU suite on the current tree, then paired A/B runs of the
# product library against build/prev (configs in ABCONFIGS).  Each GPU step
# has its own limit; the first failure ends the script.
set -o pipefail
TAG=${TAG:-rXX} bash tools/gpu_tests.sh || exit 1
for c in ${ABCONFIGS:-3 5}; do
  CONFIG=$c NAMES=prev bash tools/ab_libs.sh || exit 1
done
