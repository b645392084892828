# msd_fallback with device-picked groups + pinned work lists: MSD + large GPU tests, C5 x2 and C4 bench lines
set -o pipefail
O=gpurun_out/r03p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for w in c5 c5 c4; do
timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/$w.json 2> $O/$w.err || { echo "$w rc=$?"; tail -20 $O/$w.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/$w.json')); k=d['kernels']; print('$w', d['ms_per_step'], 'kernels', round(sum(v['ms_per_step'] for v in k.values()),2), {a: v['ms_per_step'] for a, v in k.items() if v['ms_per_step'] > 0.1})"
done
