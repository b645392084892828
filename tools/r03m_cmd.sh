# part_b FASTMAX 128 / 32 / 16 with the parallel ballot path (C5); 8192-row pass-A tiles (C3 A/B + MSD tests on that build)
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
export TMPDIR=/tmp
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03m fm128 fm32 fm16 || exit 1
bash tools/ab2.sh r03m fm128 pa8k || exit 1
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/pa8k/libsmj_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pa8k_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $O/pa8k_tests.txt; exit 1; }
tail -1 $O/pa8k_tests.txt
