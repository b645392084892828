# device-set occurrence cuts + concurrent pulls (multidev suite); C5 big-group tier: rocprof stats, size histogram, job-split threshold probe
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multidev.py tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.out; exit 1; }
tail -1 $O/tests.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python3 bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_prof.json 2> $O/c5_prof.err || { echo "prof rc=$?"; tail -5 $O/c5_prof.err; exit 1; }
rm -f $O/prof/c5_kernel_trace.csv
head -14 $O/prof/c5_kernel_stats.csv | cut -c1-150
SMJ_DEBUG_BIG=1 timeout -k 10 300 python bench.py --workload c5 --steps 1 --warmup 0 --cpu-sample 0 --cpu-mt 0 > $O/c5_dbg.json 2> $O/c5_dbg.err || { echo "dbg rc=$?"; tail -5 $O/c5_dbg.err; exit 1; }
for cfg in "131072 32768" "32768 32768" "32768 8192"; do set -- $cfg
SMJ_BG_MAX_ROWS=$1 SMJ_BG_SEG=$2 timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_$1_$2.json 2> $O/c5_$1_$2.err || { echo "c5 $cfg rc=$?"; tail -5 $O/c5_$1_$2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_$1_$2.json')); print('$cfg', d['ms_per_step'], d['kernels']['msd_big_dev'])"
done
timeout -k 10 600 python -u -m pytest tests/test_dist_gloo.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dist_tests.out 2>&1 || { echo "dist tests rc=$?"; tail -40 $O/dist_tests.out; exit 1; }
tail -1 $O/dist_tests.out
timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > $O/loop.json 2> $O/loop.err || { echo "loop rc=$?"; tail -20 $O/loop.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/loop.json')); print('loopback', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.05})"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ltrace -o loop -- python3 bench.py --loopback --steps 3 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/loop_prof.json 2> $O/loop_prof.err || { echo "ltrace rc=$?"; tail -5 $O/loop_prof.err; exit 1; }
python3 tools/trace_gaps.py $O/ltrace/loop_kernel_trace.csv --top 30 > $O/loop_gaps.txt; head -40 $O/loop_gaps.txt
