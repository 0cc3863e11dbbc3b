#!/bin/bash
# rocprofv3 evidence for the env step alone (bench.py --env-only,
# venv_step_kernel: SURVEY 8(d) K1) at config 3's env batch and at a batch
# where HBM binds, and for the GAE scan (gae_kernel, K5) in a config-3
# trainer at 1M envs: kernel trace + stats, FETCH_SIZE, WRITE_SIZE and one SQ
# pass (occupancy, wait / issue shares).  Summaries -> gpurun_out/profiles/
# <TAG>_env<N>_* with the run's env count in their _meta (bench.py cites a
# summary's traffic only for the same library, env count and shape).
#   TAG=r06c ENVS="32768 1048576" bash tools/gpu_profile_env.sh
set -o pipefail
TAG=${TAG:-rXX}
ENVS=${ENVS:-"32768 1048576"}
O=gpurun_out
mkdir -p $O/profiles
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
run_set() {  # name, meta json, bench args
  local name=$1 meta=$2; shift 2
  local D=$O/prof_${TAG}_$name
  rm -rf $D; mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run \
      -- python3 bench.py "$@" > $D/trace.log 2>&1 || { tail -5 $D/trace.log; return 1; }
  for pass in FETCH_SIZE WRITE_SIZE "$SQ"; do
    n=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $D/pmc_$n -o run \
        -- python3 bench.py "$@" > $D/pmc_$n.log 2>&1 || { tail -5 $D/pmc_$n.log; return 1; }
  done
  PMC_META="$meta" PMC_PRINT=${PRINT:-venv_step} PROFILE_OUT=$O/profiles \
      python3 tools/pmc_summary.py ${TAG}_$name $D/trace $D/pmc_FETCH_SIZE \
      $D/pmc_WRITE_SIZE $D/pmc_SQ_WAVES > $D/summary.log 2>&1 || { cat $D/summary.log; return 1; }
  cat $D/summary.log
}
for n in $ENVS; do
  run_set env$n "{\"workload\": \"env_only\", \"envs\": $n, \"bins\": 64, \"dims\": 2}" \
      --env-only --envs $n --steps 20 --warmup 2 || exit 1
done
PRINT=gae run_set c3_env1m "{\"workload\": \"config3_trainer\", \"envs\": 1048576}" \
    --envs 1048576 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
