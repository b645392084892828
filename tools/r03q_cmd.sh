# msd_fallback without the slot map: MSD + large tests, C5 line; C5 kernel-trace gaps; C3 / C5 phase stamps
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_msd.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); k=d['kernels']; print('c5', d['ms_per_step'], 'kernels', round(sum(v['ms_per_step'] for v in k.values()),2))"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c5 -o c5 -- python3 bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_trace.json 2> $O/c5_trace.err || { echo "trace rc=$?"; tail -5 $O/c5_trace.err; exit 1; }
T=$(ls $O/trace_c5/*kernel_trace.csv | head -1)
python3 tools/trace_gaps.py $T --from-kernel msd_part1 --top 30 > $O/c5_gaps.txt && head -60 $O/c5_gaps.txt
rm -f $T
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so timeout -k 10 300 python tools/msd_phases.py > $O/c3_phases.txt 2>&1 || { echo "phases rc=$?"; tail -5 $O/c3_phases.txt; exit 1; }
cat $O/c3_phases.txt
