# RCCL loopback (C3 on one GPU through smj.dist): exchange stage count K = 1, 2, 3, 4, 6, 8, two rounds
set -o pipefail
O=gpurun_out/r03zg; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for k in 2 4 3 6 8 1; do
SMJ_DIST_STAGES=$k timeout -k 10 300 python bench.py --loopback --cpu-sample 0 --cpu-mt 0 > $O/loop_k$k.$r.json 2> $O/loop_k$k.$r.err || { echo "k=$k rc=$?"; tail -20 $O/loop_k$k.$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/loop_k$k.$r.json')); print('K=$k', d['ms_per_step'], d['config'].get('exchange_stages'))"
done
done | tee $O/summary.txt
