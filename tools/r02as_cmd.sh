# device big groups wave-turn ranking, run list built once per group: targeted tests, C5 size distribution of the oversized groups, C5 timing
set -o pipefail
O=gpurun_out/r02as; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_msd.py -x -q -k "oversized or zipf or single_key or long_equal" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_big.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests_big.out; exit 1; }
tail -1 $O/tests_big.out
SMJ_DEBUG_BIG=1 timeout -k 10 300 python bench.py --workload c5 --steps 1 --warmup 0 --cpu-sample 0 --cpu-mt 0 > $O/c5dbg.json 2> $O/c5dbg.err || { echo "c5dbg rc=$?"; tail -20 $O/c5dbg.err; exit 1; }
grep "smj big" $O/c5dbg.err | sort | uniq -c | sort -k8 -n | tail -40
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print(d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.2})"
