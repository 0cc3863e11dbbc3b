#!/bin/bash
# The round's bench lines only (configs 3 with the CPU baseline, 2, 5, the
# larger-T point and the KL-PPO side lines), citing the newest committed PMC
# summaries; TAG names the round.  Each step has its own limit.
set -o pipefail
TAG=${TAG:-rXX}
O=gpurun_out
mkdir -p $O/profiles
timeout -k 10 400 python -u bench.py > $O/b3.log 2>&1 || { tail -5 $O/b3.log; exit 1; }
tail -1 $O/b3.log > $O/profiles/${TAG}_bench_config3.json
for c in 2 5; do
  timeout -k 10 400 python -u bench.py --config $c > $O/b$c.log 2>&1 || { tail -5 $O/b$c.log; exit 1; }
  tail -1 $O/b$c.log > $O/profiles/${TAG}_bench_config$c.json
done
timeout -k 10 300 python -u bench.py --rollout-steps 32 --steps 3 --warmup 1 --no-cpu-baseline > $O/bT32.log 2>&1 || { tail -5 $O/bT32.log; exit 1; }
tail -1 $O/bT32.log > $O/profiles/${TAG}_bench_config3_T32.json
for c in 3 2 5; do
  timeout -k 10 300 python -u bench.py --config $c --algo klppo --steps 5 --warmup 1 > $O/bkl$c.log 2>&1 || { tail -5 $O/bkl$c.log; exit 1; }
  tail -1 $O/bkl$c.log > $O/profiles/${TAG}_bench_config${c}_klppo.json
done
timeout -k 10 120 python -u bench.py --env-only --steps 20 --warmup 2 > $O/benv.log 2>&1 || { tail -5 $O/benv.log; exit 1; }
tail -1 $O/benv.log > $O/profiles/${TAG}_bench_envonly.json
timeout -k 10 120 python -u bench.py --env-only --envs 1048576 --steps 20 --warmup 2 --no-cpu-baseline > $O/benv1m.log 2>&1 || { tail -5 $O/benv1m.log; exit 1; }
tail -1 $O/benv1m.log > $O/profiles/${TAG}_bench_envonly_1m.json
cut -c1-200 $O/profiles/${TAG}_bench_config*.json
