# C4 on one GPU: why msd_final runs at 0.13 of peak there (kernel stats + stage stats)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02q
timeout -k 10 300 python bench.py --workload c4 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > gpurun_out/r02q/bench_c4.json 2> gpurun_out/r02q/bench_c4.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02q/prof -o run -- python bench.py --workload c4 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > gpurun_out/r02q/prof.out 2> gpurun_out/r02q/prof.err
rc=$?; rm -f gpurun_out/r02q/prof/run_kernel_trace.csv; echo rc=$rc
