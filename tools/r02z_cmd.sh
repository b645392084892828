# direct join (look-back in the staged final kernel, no msd_compact): MSD + large GPU tests, then same-box A/B
set -o pipefail
O=gpurun_out/r02z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
SMJ_DEBUG_LB=1 timeout -k 10 120 python bench.py --cpu-sample 0 --cpu-mt 0 > $O/dbg.json 2> $O/dbg.err || exit 1
tail -3 $O/dbg.err
bash tools/ab.sh r02z head lb2 lb1 lb0 || exit 1
for r in 1 2; do SMJ_DIRECT_JOIN=0 SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/lb2/libsmj_hip.so timeout -k 10 120 python bench.py --cpu-sample 0 --cpu-mt 0 > $O/nodirect.$r.json || exit 1
python3 -c "import json; d=json.load(open('$O/nodirect.$r.json')); print('nodirect', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.05})"; done | tee -a $O/ab.txt
