mkdir -p gpurun_out/r02j
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/w6o/libsmj_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02j/msd.out 2>&1 && \
bash tools/ab.sh r02j orig w4o w6o
echo rc=$? >> gpurun_out/r02j/msd.out
