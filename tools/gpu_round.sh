#!/bin/bash
# Round evidence on one box: the rocprofv3 passes of every config
# (tools/gpu_profile.sh), then the bench lines (config 3 with the CPU
# baseline, configs 2 / 5, the larger-T point) citing those summaries.  TAG
# names the round.  Each step has its own limit; the first failure ends the
# script.
set -o pipefail
TAG=${TAG:-rXX}
O=gpurun_out
mkdir -p $O/profiles
# the counters first, so that the bench lines cite this round's summaries
TAG=$TAG bash tools/gpu_profile.sh || exit 1
cp $O/profiles/${TAG}_c*_pmc_summary.json profiles/
timeout -k 10 400 python -u bench.py > $O/profiles/${TAG}_bench_config3.json.log 2>&1 || { tail -5 $O/profiles/${TAG}_bench_config3.json.log; exit 1; }
tail -1 $O/profiles/${TAG}_bench_config3.json.log > $O/profiles/${TAG}_bench_config3.json
for c in 2 5; do
  timeout -k 10 400 python -u bench.py --config $c > $O/b$c.log 2>&1 || { tail -5 $O/b$c.log; exit 1; }
  tail -1 $O/b$c.log > $O/profiles/${TAG}_bench_config$c.json
done
timeout -k 10 300 python -u bench.py --rollout-steps 32 --steps 3 --warmup 1 --no-cpu-baseline > $O/bT32.log 2>&1 || { tail -5 $O/bT32.log; exit 1; }
tail -1 $O/bT32.log > $O/profiles/${TAG}_bench_config3_T32.json
# side line: kl_ppo_learner on the config-3 shape (its split train kernel)
timeout -k 10 300 python -u bench.py --algo klppo --steps 5 --warmup 1 --no-cpu-baseline > $O/bkl.log 2>&1 || { tail -5 $O/bkl.log; exit 1; }
tail -1 $O/bkl.log > $O/profiles/${TAG}_bench_config3_klppo.json
cut -c1-400 $O/profiles/${TAG}_bench_config*.json
