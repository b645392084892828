# device big-group kernel (cap 131072 rows, large-first tickets): full GPU suite, C3 bench, C5 and C4 benches
set -o pipefail
O=gpurun_out/r02at; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
timeout -k 10 300 python bench.py --cpu-sample 0 --cpu-mt 0 > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c4.json 2> $O/c4.err || { echo "c4 rc=$?"; exit 1; }
for w in c3 c5 c4; do python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['ms_per_step'], d['value'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"; done
