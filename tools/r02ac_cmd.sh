# full GPU suite (incl. the RCCL loopback tests), bench, and the distributed path at N = 1 over RCCL loopback
set -o pipefail
O=gpurun_out/r02ac; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -2 $O/tests.out
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > $O/loopback.json 2> $O/loopback.err || { tail $O/loopback.err; exit 1; }
cat $O/bench.json; cat $O/loopback.json
