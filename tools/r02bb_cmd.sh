# group packing fused into msd_group_kernel (look-back over the published bucket group counts): MSD + large + multidev GPU tests, same-box A/B vs HEAD
set -o pipefail
O=gpurun_out/r02bb; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py tests/test_gpu_multidev.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
bash tools/ab.sh r02bb head grp1
