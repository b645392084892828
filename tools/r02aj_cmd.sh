# part_b: scalar metadata loads + unconditional stores -> the loop top waits vmcnt(4) (rows only), not vmcnt(0)
# MSD + large GPU tests, then same-box A/B: HEAD, fix1 (tn2 moved, final offsB preload), fix2 (current), pbnost (no part_b row stores)
set -o pipefail
O=gpurun_out/r02aj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
bash tools/ab.sh r02aj head fix1 fix2 pbnost && timeout -k 10 200 python3 tools/pb_ablate.py > $O/pb_ablate.txt 2>&1
