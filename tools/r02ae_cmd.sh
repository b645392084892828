# pipelined part_b (next tile gathered before this tile's stores): MSD + large GPU tests, same-box A/B vs HEAD
set -o pipefail
O=gpurun_out/r02ae; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
bash tools/ab.sh r02ae head pipe
