#!/bin/bash
# SQ counter passes over a short bench run (one pass per counter set).
#   bash tools/pmc_sq.sh            -> gpurun_out/sq_list.txt + gpurun_out/sq_*/
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 60 rocprofv3 -L > $O/sq_list.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" $O/sq_list.txt | sort -u > $O/sq_names.txt
i=0
for set in "$@"; do
  i=$((i+1))
  rm -rf $O/sq_$i
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/sq_$i -o run \
      -- python3 bench.py $ARGS > $O/sq_$i.log 2>&1 || { tail -5 $O/sq_$i.log; exit 1; }
done
python3 - "$@" <<'PY'
import csv, glob, collections, sys
for i in range(1, len(sys.argv)):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/sq_%d/**/*counter_collection.csv" % i, recursive=True):
        for r in csv.DictReader(open(f)):
            if "policy_train" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print("%-32s %16.0f  (n=%d)" % (k, sum(v) / len(v), len(v)))
PY
