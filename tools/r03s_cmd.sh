# combined-capacity final groups (<= 2048 rows of both tables): MSD + large + parity tests, then C3 / C5 A/B vs the previous kernel (old) and per-table packing (SMJ_ST_PERTABLE=1)
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ab2.sh r03s comb old || exit 1
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03s comb old || exit 1
SMJ_ST_PERTABLE=1 WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03s_pt comb || exit 1
