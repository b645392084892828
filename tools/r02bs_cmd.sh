# C4 and C5 on one GPU (partitioned mode) on HEAD: bench lines + kernel split
set -o pipefail
O=gpurun_out/r02bs; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c4.json 2> $O/c4.err || { echo "c4 rc=$?"; tail -20 $O/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5.json 2> $O/c5.err || { echo "c5 rc=$?"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
