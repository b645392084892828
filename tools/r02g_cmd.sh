mkdir -p gpurun_out/r02g
timeout -k 10 600 python -u -m pytest tests/test_gpu_multidev.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02g/multidev.out 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02g/tests.out 2>&1
echo rc=$? >> gpurun_out/r02g/tests.out
