# 255 pass-A splitters (9-bit part_a digit): full GPU suite, same-box A/B against 127 (b7), C4 stats
set -o pipefail
mkdir -p gpurun_out/r02r
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02r/tests.out 2>&1 && \
bash tools/ab.sh r02r b7 b8 && \
timeout -k 10 300 python bench.py --workload c4 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > gpurun_out/r02r/bench_c4.json 2> gpurun_out/r02r/bench_c4.err
echo rc=$?
