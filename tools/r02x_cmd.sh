# 32-bit pass-B digit + materialised scan prefixes in the final stage (72 VGPRs): MSD tests, A/B vs HEAD (r3)
set -o pipefail
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 && \
bash tools/ab.sh r02x r3 s32
echo rc=$?
