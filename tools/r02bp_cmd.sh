# 12-byte pass-A rows: MSD GPU tests on the narrow build, then same-box A/B narrow vs wide (SMJ_NARROW_A=0)
set -o pipefail
O=gpurun_out/r02bp; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_msd.out 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests_msd.out; exit 1; }
tail -1 $O/tests_msd.out
bash tools/ab.sh r02bp narrow wide
