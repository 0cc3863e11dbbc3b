#!/bin/bash
# Ad-hoc GPU check: XCD-aware split order of the value net's weight-gradient
# kernel -- bit-identity and parity tests, A/B, FETCH_SIZE of the kernel.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_value.py tests/test_gpu_parity.py tests/test_gpu_model_api.py > $O/chk_tests.txt 2>&1 || { tail -30 $O/chk_tests.txt; exit 1; }
tail -2 $O/chk_tests.txt
for c in 5 3; do CFG=$c ROUNDS=2 bash tools/ab_lib.sh build/base/libxylo_hip.so || exit 1; done
for c in 5 3; do
  ARGS="--config $c --steps 3 --warmup 1 --no-cpu-baseline"
  for v in product base; do
    rm -rf $O/fx_${v}_$c
    if [ $v = base ]; then export XH_LIB_PATH=build/base/libxylo_hip.so; else unset XH_LIB_PATH; fi
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fx_${v}_$c -o run -- python3 bench.py $ARGS > $O/fx_${v}_$c.log 2>&1 || { tail -5 $O/fx_${v}_$c.log; exit 1; }
    rm -rf $O/tx_${v}_$c
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tx_${v}_$c -o run -- python3 bench.py $ARGS > $O/tx_${v}_$c.log 2>&1 || { tail -5 $O/tx_${v}_$c.log; exit 1; }
  done
done
unset XH_LIB_PATH
python3 - <<'PY'
import csv, glob, collections
for c in ("5", "3"):
  for v in ("product", "base"):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/fx_%s_%s/**/*counter_collection.csv" % (v, c), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE" and "mlp3" in r["Kernel_Name"]:
                agg[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
    dur = {}
    for f in glob.glob("gpurun_out/tx_%s_%s/**/*kernel_stats.csv" % (v, c), recursive=True):
        for r in csv.DictReader(open(f)):
            if "mlp3" in r["Name"]: dur[r["Name"][:40]] = float(r["AverageNs"]) / 1e3
    for k, x in agg.items():
        print(c, v, k, "FETCH x2 %.1f MB" % (2 * sum(x) / len(x) * 1024 / 1e6), "avg %.1f us" % dur.get(k, -1))
PY
