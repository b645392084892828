# giant-job size with the 65536-row threshold: SMJ_BG_SEG 32768 (default) / 16384 / 65536 on C5
set -o pipefail
O=gpurun_out/r03zc; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for g in 32768 16384 65536; do
SMJ_BG_SEG=$g timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_seg$g.$r.json 2> $O/c5_seg$g.$r.err || { echo "seg $g rc=$?"; tail -20 $O/c5_seg$g.$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_seg$g.$r.json')); print('c5 seg $g', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if k in ('msd_big_dev', 'msd_final', 'msd_compact')})"
done; done | tee $O/ab_seg.txt
