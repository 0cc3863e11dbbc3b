set -o pipefail
O=gpurun_out; mkdir -p $O/profiles
rm -f $O/global_sums.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_global.py tests/test_gpu_tensor.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/profiles/r05b_gpu_tests.txt 2>&1; rc=$?
tail -8 $O/profiles/r05b_gpu_tests.txt
cp $O/global_sums.jsonl $O/profiles/r05b_global_sums.jsonl 2>/dev/null
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --env-only --steps 50 --warmup 5 > $O/profiles/r05b_bench_envonly.json 2> $O/envonly.err || { tail -5 $O/envonly.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > $O/profiles/r05b_bench_config3.json 2> $O/b3.err || { tail -5 $O/b3.err; exit 1; }
cut -c1-700 $O/profiles/r05b_bench_envonly.json $O/profiles/r05b_bench_config3.json
timeout -k 10 120 ./build/probe_sp > $O/profiles/r05b_probe_specialize.txt 2>&1 || { tail -5 $O/profiles/r05b_probe_specialize.txt; exit 1; }
cat $O/profiles/r05b_probe_specialize.txt
