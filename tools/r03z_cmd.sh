# one-pass partition: staging overlapped with wave 0's look-back (head) vs after it (prev): large tests, C4 / C5 A/B
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
WORKLOAD=c4 STEPS=3 WARMUP=1 bash tools/ab2.sh r03z head prev || exit 1
WORKLOAD=c5 STEPS=3 WARMUP=1 bash tools/ab2.sh r03z head prev || exit 1
