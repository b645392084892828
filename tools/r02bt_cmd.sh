# part_b: heavy-key buckets skip counting and ranking. MSD + large GPU tests, then same-box C5 and C3 A/B
set -o pipefail
O=gpurun_out/r02bt; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.out; exit 1; }
tail -1 $O/tests.out
for r in 1 2; do for v in onekey nokey; do
  SMJ_LIB=$GRAFT_REPO_ROOT/pim-sort-merge-join_amd/lib/variants/$v/libsmj_hip.so timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_$v.$r.json 2> $O/c5_$v.$r.err || { echo "c5 $v rc=$?"; tail -20 $O/c5_$v.$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.$r.json')); print('c5 $v', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
done; done | tee $O/c5_ab.txt
bash tools/ab.sh r02bt_c3 onekey nokey
