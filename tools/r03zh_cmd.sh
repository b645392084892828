# final validation of the session on HEAD (after the tile-size switches): full GPU suite + smoke; C3 bench line (CPU baselines); C4 / C5 lines; C3 + C5 rocprof kernel stats; loopback
set -o pipefail
O=gpurun_out/r03zh; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -20 $O/c3.err; exit 1; }
for w in c5 c4; do
timeout -k 10 400 python bench.py --workload $w --steps 5 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/$w.json 2> $O/$w.err || { echo "$w rc=$?"; tail -20 $O/$w.err; exit 1; }
done
for w in c3 c5 c4; do
python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.1})"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_prof.json 2> $O/c5_prof.err || { echo "prof c5 rc=$?"; tail -5 $O/c5_prof.err; exit 1; }
rm -f $O/prof_c5/c5_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/c3_prof.json 2> $O/c3_prof.err || { echo "prof c3 rc=$?"; tail -5 $O/c3_prof.err; exit 1; }
rm -f $O/prof_c3/c3_kernel_trace.csv
timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > $O/loop.json 2> $O/loop.err || { echo "loop rc=$?"; tail -20 $O/loop.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/loop.json')); print('loopback', d['ms_per_step'])"
