# per-table join lookups back to 2 per thread: MSD tests; C3 A/B vs old; C4 with 1.0e8-row parts vs 1.5e8
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ab2.sh r03u new old || exit 1
WORKLOAD=c4 STEPS=3 WARMUP=1 bash tools/ab2.sh r03u new || exit 1
SMJ_PART_ROWS=1e8 WORKLOAD=c4 STEPS=3 WARMUP=1 bash tools/ab2.sh r03u_p1e8 new || exit 1
SMJ_PART_ROWS=1e8 WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03u_p1e8 new || exit 1
