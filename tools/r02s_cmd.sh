# 256 dup-aware pass-A buckets (8-bit digit): full GPU suite, A/B vs the 9-bit build (b9), C4 + C5, kernel stats, phase stamps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 && \
bash tools/ab.sh r02s b9 n8 && \
timeout -k 10 300 python bench.py --workload c4 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/bench_c4.json 2> $O/bench_c4.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/bench_c5.json 2> $O/bench_c5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/prof.out 2> $O/prof.err && \
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/st8/libsmj_hip.so timeout -k 10 300 python tools/msd_phases.py > $O/phases.txt 2> $O/phases.err
rc=$?; rm -f $O/prof/run_kernel_trace.csv; echo rc=$rc
