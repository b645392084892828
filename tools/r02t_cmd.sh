# runs_apply as wave-per-bucket (coalesced list stores): MSD GPU tests, A/B vs HEAD (r0), final-stage ablation
set -o pipefail
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 && \
bash tools/ab.sh r02t r0 n1 && \
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/abl/libsmj_hip.so timeout -k 10 300 python tools/final_ablate.py > $O/final_ablate.txt 2> $O/final_ablate.err
echo rc=$?
