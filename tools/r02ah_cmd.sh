# part_b: next-next tile info loaded at the loop top (no vmcnt(0) between the next tile's gathers and this tile's stores);
# final stage: offsB of group li + 1 preloaded in iteration li - 1.  MSD + large GPU tests, then same-box A/B vs HEAD
set -o pipefail
O=gpurun_out/r02ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
bash tools/ab.sh r02ah head fix1
