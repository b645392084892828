# part_b: per-quad sub-bucket counts (fix-up over a quad's group), popcount run lookup: GPU suite, A/B vs HEAD (r1)
set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.out 2>&1 && \
bash tools/ab.sh r02v r1 pq
echo rc=$?
