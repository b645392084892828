# batched oversized-group fallback: its GPU tests, C5 bench; fused part_a / 512-segment A/B on C3
set -o pipefail
mkdir -p gpurun_out/r02o
timeout -k 10 300 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02o/tests_msd.out 2>&1 && \
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r02o/bench_c5.json 2> gpurun_out/r02o/bench_c5.err && \
bash tools/ab.sh r02o_ab head fused seg512
echo rc=$? >> gpurun_out/r02o/tests_msd.out
