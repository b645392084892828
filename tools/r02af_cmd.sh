# pipelined part_b, next run list marked from registers (one barrier fewer per tile): MSD + large GPU tests, A/B vs HEAD and the first pipelined version
set -o pipefail
O=gpurun_out/r02af; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
bash tools/ab.sh r02af head pipe pipe2
