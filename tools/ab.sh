#!/bin/bash
# tools/ab.sh TAG variant... -- same-box A/B of library variants
# (tools/build_variant.sh), two rounds, each run under its own limit.
# BENCH_ARGS: extra bench.py flags (e.g. "--workload c5 --steps 5 --warmup 2").
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
i=2
while [ -e "$OUT" ]; do OUT=$ROOT/gpurun_out/${TAG}_$i; i=$((i + 1)); done
mkdir -p $OUT
for r in 1 2; do
  for v in "$@"; do
    SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/$v/libsmj_hip.so timeout -k 10 300 python $ROOT/bench.py --cpu-sample 0 --cpu-mt 0 ${BENCH_ARGS:-} > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { echo "$v failed rc=$?"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/$v.$r.json')); print('$v', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.05})"
  done
done | tee $OUT/ab.txt
