# session 2 start: full GPU suite + smoke on HEAD (bbd19e8 changed smj_msd.hip after r03i); C3 bench line (with CPU baselines), C5 and C4 lines
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
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
# part_b's ballot path on per-wave counters (SMJ_PB_SLOWPAR, now default) vs waves in turn; FASTMAX 32 with it
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03l_ab spar sser spar32 || exit 1
# part_b rows stored straight from registers (no LDS staging) vs staged: C3
bash tools/ab2.sh r03l_ab spar pbdirect || exit 1
