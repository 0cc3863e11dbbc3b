#!/bin/bash
# SQ counters of the config-3 train kernel under several XH_TRAIN_KERNEL
# values (diagnostic A/B, one rocprofv3 pass per counter set):
#   bash tools/pmc_ab.sh default split8wp
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/sq_list.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" $O/sq_list.txt | sort -u > $O/sq_names.txt
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"
      "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE")
for k in "$@"; do
  if [ $k = default ]; then unset XH_TRAIN_KERNEL; A=""; else export XH_TRAIN_KERNEL=$k; A="--allow-kernel-override"; fi
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    for c in $set; do grep -qx $c $O/sq_names.txt || { echo "no counter $c"; exit 1; }; done
    rm -rf $O/pab_${k}_$i
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pab_${k}_$i -o run \
        -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $A > $O/pab_${k}_$i.log 2>&1 || { tail -5 $O/pab_${k}_$i.log; exit 1; }
  done
done
python3 - "$@" <<'PY'
import csv, glob, collections, sys
for k in sys.argv[1:]:
    print("==", k)
    for i in (1, 2):
        agg = collections.defaultdict(list)
        for f in glob.glob("gpurun_out/pab_%s_%d/**/*counter_collection.csv" % (k, i), recursive=True):
            for r in csv.DictReader(open(f)):
                if "policy_train" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for n, v in sorted(agg.items()):
            print("%-32s %16.0f  (n=%d)" % (n, sum(v) / len(v), len(v)))
PY
