#!/bin/bash
# tools/ab.sh TAG variant... -- same-box A/B of library variants (WORKLOAD=c3|c4|c5)
# (tools/build_variant.sh) on the C3 bench, two rounds, each under its own limit.
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2; do
  for v in "$@"; do
    SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/$v/libsmj_hip.so timeout -k 10 300 python $ROOT/bench.py --workload ${WORKLOAD:-c3} --steps ${STEPS:-10} --warmup ${WARMUP:-3} --cpu-sample 0 --cpu-mt 0 > $OUT/${WORKLOAD:-c3}_$v.$r.json 2> $OUT/${WORKLOAD:-c3}_$v.$r.err || { echo "$v failed rc=$?"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/${WORKLOAD:-c3}_$v.$r.json')); print('$v', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.05})"
  done
done | tee $OUT/ab_${WORKLOAD:-c3}.txt
