# C5 one step per timing-ablation build of the device big-group tiers (output invalid except bg0): msd_big_dev ms
O=gpurun_out/r02bi; mkdir -p $O
for v in bg0 bg1 bg2 bg4 bg3; do
  SMJ_LIB=$GRAFT_REPO_ROOT/pim-sort-merge-join_amd/lib/variants/$v/libsmj_hip.so timeout -k 10 200 python bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 --cpu-mt 0 > $O/$v.json 2> $O/$v.err
  echo "$v rc=$?"; python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['ms_per_step'], d['kernels'].get('msd_big_dev', {}).get('ms_per_step'))" 2>/dev/null
done
