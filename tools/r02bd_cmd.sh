# recorded launch sequences replayed as HIP graphs: the replay test + MSD/large/parity GPU tests, then same-box A/B (HEAD vs graph), both benches timing unprofiled steps
set -o pipefail
O=gpurun_out/r02bd; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_msd.py -x -v -k "replay" --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests_replay.out 2>&1 || { echo "replay rc=$?"; tail -40 $O/tests_replay.out; exit 1; }
grep -c PASSED $O/tests_replay.out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.out; exit 1; }
tail -1 $O/tests.out
bash tools/ab.sh r02bd head graph
