# one-pass partition (msd_part1_kernel, default) vs the counting partition (SMJ_PART1=0): large-mode GPU tests, C4/C5 A/B
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/large_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/large_tests.txt; exit 1; }
tail -1 $O/large_tests.txt
for r in 1 2; do for w in c4 c5; do for v in 1 0; do
SMJ_PART1=$v timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/${w}_p$v.$r.json 2> $O/${w}_p$v.$r.err || { echo "$w p$v rc=$?"; tail -20 $O/${w}_p$v.$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${w}_p$v.$r.json')); print('$w part1=$v', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.1})"
done; done; done
