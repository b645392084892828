# loopback (one-rank RCCL group) C3 step on HEAD: bench line + kernel trace gaps
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > $O/loop.json 2> $O/loop.err || { echo "loop rc=$?"; tail -20 $O/loop.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/loop.json')); print('loopback', d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o loop -- python3 bench.py --loopback --steps 3 --warmup 2 --cpu-sample 0 --cpu-mt 0 > $O/loop_trace.json 2> $O/loop_trace.err || { echo "trace rc=$?"; tail -5 $O/loop_trace.err; exit 1; }
T=$(ls $O/trace/*kernel_trace.csv | head -1)
python3 tools/trace_steps.py $T > $O/steps.txt 2>&1; head -80 $O/steps.txt
python3 tools/trace_gaps.py $T --top 20 > $O/gaps.txt && head -45 $O/gaps.txt
