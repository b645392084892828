# msd parity on the new final-stage pipeline, then same-box A/B and stamps
mkdir -p gpurun_out/r02h
timeout -k 10 600 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02h/msd.out 2>&1 && \
bash tools/ab.sh r02h orig pipe && \
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so timeout -k 10 120 python tools/msd_phases.py > gpurun_out/r02h/phases.txt 2>&1
echo rc=$? >> gpurun_out/r02h/msd.out
