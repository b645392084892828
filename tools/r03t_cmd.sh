# staged kernel templated on the group layout (per-table for balanced tables, combined for skewed ones): MSD tests in both forced modes + large + parity; C3 / C5 A/B vs the round's previous kernel (old)
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
SMJ_ST_COMBINED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_comb1.txt 2>&1 || { echo "comb1 tests rc=$?"; tail -40 $O/tests_comb1.txt; exit 1; }
tail -1 $O/tests_comb1.txt
SMJ_ST_COMBINED=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_comb0.txt 2>&1 || { echo "comb0 tests rc=$?"; tail -40 $O/tests_comb0.txt; exit 1; }
tail -1 $O/tests_comb0.txt
bash tools/ab2.sh r03t new old || exit 1
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03t new old mr64 || exit 1
