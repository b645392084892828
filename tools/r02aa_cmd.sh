# 16-B join-slot stores in the staged final kernel: MSD tests, same-box A/B vs HEAD, then PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the current build
set -o pipefail
O=gpurun_out/r02aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
bash tools/ab.sh r02aa head j16 pa1 pa2w6 || exit 1
bash tools/gpu_run.sh r02aa pmcf pmcw pmcsq
