# one-pass partition tile 4096 (2 WG/CU) vs 3072 rows (3 WG/CU), both with the per-slot part array: large tests on p6; C4 / C5 A/B (two rounds); pass-A 3072-row tiles (pa6): msd + staged tests, C3 A/B
set -o pipefail
O=gpurun_out/r03zf; mkdir -p $O
export TMPDIR=/tmp
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/p6/libsmj_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_p6.txt 2>&1 || { echo "tests p6 rc=$?"; tail -40 $O/tests_p6.txt; exit 1; }
tail -1 $O/tests_p6.txt
WORKLOAD=c4 STEPS=3 WARMUP=1 bash tools/ab2.sh r03zf p8 p6 || exit 1
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03zf p8 p6 || exit 1
# pass-A tile 3072 rows (3 WG/CU) vs 4096: msd + staged tests on pa6, C3 A/B
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/pa6/libsmj_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_pa6.txt 2>&1 || { echo "tests pa6 rc=$?"; tail -40 $O/tests_pa6.txt; exit 1; }
tail -1 $O/tests_pa6.txt
WORKLOAD=c3 STEPS=10 WARMUP=3 bash tools/ab2.sh r03zf p8 pa6 || exit 1
