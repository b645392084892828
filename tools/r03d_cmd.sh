# resident_blocks cache per kernel (C3 check); loopback with the private compute stream (trace); big-group timing by size class
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --cpu-sample 0 --cpu-mt 0 > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -20 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.05})"
timeout -k 10 600 python -u -m pytest tests/test_dist_gloo.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dist_tests.out 2>&1 || { echo "dist tests rc=$?"; tail -40 $O/dist_tests.out; exit 1; }
tail -1 $O/dist_tests.out
timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > $O/loop.json 2> $O/loop.err || { echo "loop rc=$?"; tail -20 $O/loop.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/loop.json')); print('loopback', d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ltrace -o loop -- python3 bench.py --loopback --steps 3 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/loop_prof.json 2> $O/loop_prof.err || { echo "ltrace rc=$?"; tail -5 $O/loop_prof.err; exit 1; }
SMJ_LIB=pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so SMJ_DEBUG_BIG=1 timeout -k 10 300 python tools/big_times.py > $O/big_times.json 2> $O/big_times.err || { echo "big rc=$?"; tail -5 $O/big_times.err; exit 1; }
cat $O/big_times.json
