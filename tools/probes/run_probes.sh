#!/bin/bash
# Run the micro-probes on the box (each step under its own time limit).
set -o pipefail
mkdir -p gpurun_out/probes
export TMPDIR=/tmp
timeout -k 10 120 ./build/probe_il > gpurun_out/probes/interleave.txt 2>&1 || exit 1
cat gpurun_out/probes/interleave.txt
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/probes/$c
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/probes/$c -o run -- ./build/probe_fetch > gpurun_out/probes/$c.log 2>&1 || { tail -5 gpurun_out/probes/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/probes/%s/**/*counter_collection.csv" % c, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                agg[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(c, "%-60s %14.0f KB" % (k, sum(v) / len(v)))
PY
