# in-LDS stable LSD for equal-key runs over 32 (no radix-tier hand-over): GPU suite, A/B vs HEAD (r2), C5 bench
set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 && \
bash tools/ab.sh r02w r2 lsd && \
timeout -k 10 300 python bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/bench_c5.json 2> $O/bench_c5.err
echo rc=$?
