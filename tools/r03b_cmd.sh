# staged multi-chunk parity + MSD/large suites (giant-job buffer sizing), H2D overlap on HEAD, C3 + C5 bench lines
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.out; exit 1; }
tail -1 $O/tests.out
timeout -k 10 300 python tools/h2d_overlap.py > $O/h2d.json 2> $O/h2d.err || { echo "h2d rc=$?"; tail -20 $O/h2d.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-sample 0 --cpu-mt 0 > $O/c3.json 2> $O/c3.err || { echo "c3 rc=$?"; tail -20 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.05})"
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['ms_per_step'], d['roofline'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
