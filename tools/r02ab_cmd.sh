# RCCL transport of smj.dist in loopback mode on one GPU (nccl backend, world 1): the new GPU tests + the dist GPU tests
set -o pipefail
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist_gloo.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dist.out 2>&1; rc=$?
tail -15 $O/dist.out; exit $rc
