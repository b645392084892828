# line-aligned pass-A bucket runs (8-row padding, packed offsA starts): full GPU suite, then same-box A/B vs HEAD and fix2 (no padding)
set -o pipefail
O=gpurun_out/r02ak; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
bash tools/ab.sh r02ak head fix2 pad
