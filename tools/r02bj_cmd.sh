# big-group passes with more rows in flight (count: 4 chunks per thread; rows: next chunk prefetched): oversized + MSD/large GPU tests, C5
set -o pipefail
O=gpurun_out/r02bj; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_msd.py -x -v -k "oversized" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_big.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests_big.out; exit 1; }
grep -c PASSED $O/tests_big.out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
