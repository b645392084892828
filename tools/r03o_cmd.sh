# persistent one-pass partition (next tile's rows in flight during the look-back) vs one tile per workgroup: large tests + C4 A/B; bg_count aggregation A/B on C5
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/large_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/large_tests.txt; exit 1; }
tail -1 $O/large_tests.txt
WORKLOAD=c4 STEPS=3 WARMUP=1 bash tools/ab2.sh r03o head p1np || exit 1
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03o head noagg || exit 1
