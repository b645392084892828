# segment-record virtual part_a + block-table big-group lookups: MSD + large suites; C3, C4, C5; big-group times
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.out; exit 1; }
tail -1 $O/tests.out
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c4.json 2> $O/c4.err || { echo "c4 rc=$?"; tail -20 $O/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['ms_per_step'], d['roofline'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
SMJ_LIB=pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so SMJ_DEBUG_BIG=1 timeout -k 10 300 python tools/big_times.py > $O/big_times.json 2> $O/big_times.err || { echo "big rc=$?"; tail -5 $O/big_times.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/big_times.json')); print(d['msd_big_dev_ms'], d['phases'], {k: v['cycles_per_group'] for k, v in d['classes'].items()})"
timeout -k 10 300 python bench.py --cpu-sample 0 --cpu-mt 0 > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -20 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['ms_per_step'])"
SMJ_LIB=pim-sort-merge-join_amd/lib/variants/bounds/libsmj_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/bounds_tests.out 2>&1 || { echo "bounds tests rc=$?"; tail -40 $O/bounds_tests.out; exit 1; }
tail -1 $O/bounds_tests.out
