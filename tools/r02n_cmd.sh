# huge-page results: H2D/D2H buckets again; C4 / C5 single-GPU bench lines; full GPU suite
set -o pipefail
mkdir -p gpurun_out/r02n
timeout -k 10 600 python tools/h2d_overlap.py > gpurun_out/r02n/h2d_overlap.json 2> gpurun_out/r02n/h2d_overlap.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/r02n/bench_c4.json 2> gpurun_out/r02n/bench_c4.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r02n/bench_c5.json 2> gpurun_out/r02n/bench_c5.err && \
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02n/tests.out 2>&1
echo rc=$? >> gpurun_out/r02n/tests.out
