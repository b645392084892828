# msd_runs_seg / msd_runs_apply over both tables in one launch each: MSD GPU tests, same-box A/B vs HEAD (3 rounds)
set -o pipefail
O=gpurun_out/r02az; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
bash tools/ab.sh r02az head runs1 && bash tools/ab.sh r02az2 head runs1
