# giant-group job size sweep on C5 (SMJ_BG_SEG), then same-box C3 A/B HEAD vs giant
O=gpurun_out/r02aw; mkdir -p $O
for seg in 16384 32768 65536; do
  SMJ_BG_SEG=$seg timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_$seg.json 2> $O/c5_$seg.err || { echo "c5 $seg rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$seg.json')); print('seg $seg', d['ms_per_step'], d['kernels']['msd_final']['ms_per_step'])"
done
bash tools/ab.sh r02aw head giant
