#!/bin/bash
# Diagnostic SQ counter passes of a bench configuration's kernels for a
# list of libraries (product and XH_LIB_PATH variants): wave-cycle
# breakdown (waits, active VALU / LDS / misc), instruction fetch and LDS
# queue levels.  Prints per-kernel means per pass for the kernels whose name
# contains one of the KSUB substrings (default: the train kernel).
#   LIBS="dependence_free_rl_amd/libxylo_hip.so build/abl2/libxylo_hip.so" bash tools/pmc_diag.sh
#   CONFIG=5 KSUB="vnet_forward vnet_backward" bash tools/pmc_diag.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P2="SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_INSTS"
P3="SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
n=0
for lib in ${LIBS:-dependence_free_rl_amd/libxylo_hip.so}; do
  n=$((n+1))
  for p in 1 2 3; do
    eval pc=\$P$p
    D=gpurun_out/pmcdiag_${n}_$p
    rm -rf $D
    XH_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $pc --output-format csv -d $D -o run \
      -- python3 bench.py --config ${CONFIG:-3} --steps 2 --warmup 1 --no-cpu-baseline > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  done
  KSUB="${KSUB:-policy_train}" python3 - "$lib" $n <<'PY'
import csv, glob, os, sys, collections
lib, n = sys.argv[1], sys.argv[2]
subs = os.environ["KSUB"].split()
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in (1, 2, 3):
    for f in glob.glob("gpurun_out/pmcdiag_%s_%d/**/*counter_collection.csv" % (n, p), recursive=True):
        for r in csv.DictReader(open(f)):
            for sub in subs:
                if sub in r["Kernel_Name"]:
                    agg[sub][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(lib)
for sub in subs:
    print(" ", sub)
    for k in sorted(agg[sub]):
        v = agg[sub][k]
        print("    %-28s %16.0f" % (k, sum(v) / len(v)))
PY
done
