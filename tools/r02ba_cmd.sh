# the oversized-group tests incl. one table alone (smj_dev_select_sort)
set -o pipefail
O=gpurun_out/r02ba; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_msd.py -x -v -k "oversized" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.out; exit 1; }
grep -c PASSED $O/tests.out
