# staged final kernel: equal-key run limit for the transposition rounds (32 / 16 / 8; longer runs take the in-LDS LSD), C5 and C3 same-box A/B
set -o pipefail
O=gpurun_out/r02bx; mkdir -p $O
for r in 1 2; do for v in mr32 mr16 mr8; do
  SMJ_LIB=$GRAFT_REPO_ROOT/pim-sort-merge-join_amd/lib/variants/$v/libsmj_hip.so timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/c5_$v.$r.json 2> $O/c5_$v.$r.err || { echo "c5 $v rc=$?"; tail -20 $O/c5_$v.$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.$r.json')); print('c5 $v', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.3})"
done; done | tee $O/c5_ab.txt
bash tools/ab.sh r02bx_c3 mr32 mr16 mr8
