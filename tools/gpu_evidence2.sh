#!/bin/bash
# A round's second evidence call: the env-step / GAE counter passes
# (tools/gpu_profile_env.sh), their summaries put beside the trainer ones in
# profiles/ (so the env-only lines cite them), then every bench line
# (tools/gpu_benches.sh).  TAG names the round.
set -o pipefail
TAG=${TAG:-rXX}
O=gpurun_out
TAG=$TAG bash tools/gpu_profile_env.sh > $O/${TAG}_profenv.log 2>&1 || { tail -20 $O/${TAG}_profenv.log; exit 1; }
cp $O/profiles/${TAG}_env*_pmc_summary.json $O/profiles/${TAG}_c3_env1m_pmc_summary.json profiles/
TAG=$TAG bash tools/gpu_benches.sh
