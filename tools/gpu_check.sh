#!/bin/bash
# Ad-hoc GPU check: XCD-aware work order of the 128-bin and 32-bin train
# kernels -- parity cases, A/B against build/base, FETCH_SIZE of both.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_depth.py tests/test_gpu_shards.py tests/test_gpu_scale.py -k "b128 or b32 or c5 or c2 or 128 or 32" > $O/chk_tests.txt 2>&1 || { tail -30 $O/chk_tests.txt; exit 1; }
tail -2 $O/chk_tests.txt
for c in 5 2; do CFG=$c ROUNDS=2 bash tools/ab_lib.sh build/base/libxylo_hip.so || exit 1; done
for c in 5 2; do
  ARGS="--config $c --steps 3 --warmup 1 --no-cpu-baseline"
  for v in product base; do
    rm -rf $O/fx_${v}_$c
    if [ $v = base ]; then export XH_LIB_PATH=build/base/libxylo_hip.so; else unset XH_LIB_PATH; fi
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fx_${v}_$c -o run -- python3 bench.py $ARGS > $O/fx_${v}_$c.log 2>&1 || { tail -5 $O/fx_${v}_$c.log; exit 1; }
  done
done
unset XH_LIB_PATH
python3 - <<'PY'
import csv, glob, collections
for c in ("5", "2"):
  for v in ("product", "base"):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/fx_%s_%s/**/*counter_collection.csv" % (v, c), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE" and "policy_train" in r["Kernel_Name"]:
                agg[r["Kernel_Name"][:50]].append(float(r["Counter_Value"]))
    for k, x in agg.items():
        print(c, v, k, "FETCH_SIZE x2 = %.2f MB" % (2 * sum(x) / len(x) * 1024 / 1e6))
PY
