# giant groups split into jobs (msd_giant_count/scatter/join): targeted tests (incl. the job split at small thresholds), MSD + large tests, C5 + C3 benches
set -o pipefail
O=gpurun_out/r02av; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_msd.py -x -v -k "oversized or zipf or single_key" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_big.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests_big.out; exit 1; }
grep -c PASSED $O/tests_big.out
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
SMJ_DEBUG_BIG=1 timeout -k 10 300 python bench.py --workload c5 --steps 1 --warmup 0 --cpu-sample 0 --cpu-mt 0 > $O/c5dbg.json 2> $O/c5dbg.err || { echo "c5dbg rc=$?"; tail -20 $O/c5dbg.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail -20 $O/c5.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-sample 0 --cpu-mt 0 > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; exit 1; }
for w in c5 c3; do python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.2})"; done
