# one-pass partition tile 4096 (2 WG/CU) vs 3072 (3 WG/CU) vs 2048 rows (4 WG/CU): large tests on p6 / p4; C4 / C5 A/B
set -o pipefail
O=gpurun_out/r03ze; mkdir -p $O
export TMPDIR=/tmp
for v in p6 p4; do
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/$v/libsmj_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_$v.txt 2>&1 || { echo "tests $v rc=$?"; tail -40 $O/tests_$v.txt; exit 1; }
tail -1 $O/tests_$v.txt
done
WORKLOAD=c4 STEPS=3 WARMUP=1 bash tools/ab2.sh r03ze p8 p6 p4 || exit 1
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03ze p8 p6 p4 || exit 1
