#!/bin/bash
# The GPU suite (tools/gpu_tests.sh), then the env-only and config-3 bench
# lines, evidence under gpurun_out/profiles/<TAG>_*.  Each GPU step has its
# own limit; the first failure ends the script.
set -o pipefail
TAG=${TAG:-rXX}
O=gpurun_out
mkdir -p $O/profiles
rm -f $O/global_sums.jsonl $O/sampling_agreement.jsonl $O/shard_sums.jsonl
TAG=$TAG bash tools/gpu_tests.sh; rc=$?
for f in global_sums sampling_agreement shard_sums; do
  [ -f $O/$f.jsonl ] && cp $O/$f.jsonl $O/profiles/${TAG}_$f.jsonl
done
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --env-only --steps 50 --warmup 5 \
    > $O/profiles/${TAG}_bench_envonly.json 2> $O/envonly.err || { tail -5 $O/envonly.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline \
    > $O/profiles/${TAG}_bench_config3.json 2> $O/b3.err || { tail -5 $O/b3.err; exit 1; }
cut -c1-600 $O/profiles/${TAG}_bench_envonly.json $O/profiles/${TAG}_bench_config3.json
