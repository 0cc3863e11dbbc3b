#!/bin/bash
# rocprofv3 evidence for every bench configuration, one pass per counter set
# (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, two SQ passes for the MFMA
# utilisation).  Summaries land in gpurun_out/profiles/<TAG>_c<cfg>_*.
#   TAG=r02a CONFIGS="3 2 5" bash tools/gpu_profile.sh
#   TAG=r04zkl CONFIGS=3 EXTRA="--algo klppo" bash tools/gpu_profile.sh  (a side line)
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${TAG:-rXX}
CONFIGS=${CONFIGS:-"3 2 5"}
O=gpurun_out
mkdir -p $O/profiles
export TMPDIR=/tmp
SQ1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F32"
for c in $CONFIGS; do
  ARGS="--config $c --steps 3 --warmup 1 --no-cpu-baseline $EXTRA"
  D=$O/prof_${TAG}_c$c
  rm -rf $D; mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run \
      -- python3 bench.py $ARGS > $D/trace.log 2>&1 || { tail -5 $D/trace.log; exit 1; }
  for pass in FETCH_SIZE WRITE_SIZE "$SQ1" "$SQ2"; do
    n=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $D/pmc_$n -o run \
        -- python3 bench.py $ARGS > $D/pmc_$n.log 2>&1 || { tail -5 $D/pmc_$n.log; exit 1; }
  done
  PROFILE_OUT=$O/profiles python3 tools/pmc_summary.py ${TAG}_c$c $D/trace \
      $D/pmc_FETCH_SIZE $D/pmc_WRITE_SIZE $D/pmc_SQ_VALU_MFMA_BUSY_CYCLES \
      $D/pmc_SQ_WAIT_ANY > $D/summary.log 2>&1 || { cat $D/summary.log; exit 1; }
  head -40 $D/summary.log
done
