# new default final kernel: parity, C5 through smj.dist with 8 ranks on one GPU, bench, rocprof
set -o pipefail
mkdir -p gpurun_out/r02l
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py tests/test_gpu_multidev.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02l/tests.out 2>&1 && \
timeout -k 10 600 python -u tools/dist_c5.py --ranks 8 -o gpurun_out/r02l/dist_c5.json > gpurun_out/r02l/dist_c5.log 2>&1 && \
bash tools/gpu_run.sh r02l quick prof
echo rc=$? >> gpurun_out/r02l/tests.out
