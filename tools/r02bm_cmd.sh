# round validation on HEAD: full GPU suite, smoke, default bench, rocprof kernel stats of the bench
set -o pipefail
O=gpurun_out/r02bm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/prof_bench.json 2> $O/prof.err || { echo "prof rc=$?"; tail -5 $O/prof.err; exit 1; }
rm -f $O/prof/run_kernel_trace.csv
head -5 $O/prof/run_kernel_stats.csv
