# C5 one step under rocprofv3 --kernel-trace --stats: the device big-group kernel's own time
set -o pipefail
O=gpurun_out/r02bg; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload c5 --steps 1 --warmup 0 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "rc=$?"; tail -5 $O/c5.err; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print(f\"{r['Name'][:60]:60s} {r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f} max_us={float(r['MaxNs'])/1e3:9.1f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f}\")
" | head -30
rm -f $O/prof/run_kernel_trace.csv
