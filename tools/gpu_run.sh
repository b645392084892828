#!/bin/bash
# tools/gpu_run.sh TAG [steps...] -- the one parameterised GPU-box runner
# (replaces the per-run tools/rNN_cmd.sh records of rounds 2-3; the commands
# each run used are in git history and its outputs under profiles/).
#
#   gpurun -- 'bash tools/gpu_run.sh r04a tests smoke c3 c4 c5 loop prof'
#
# Output goes to gpurun_out/TAG; if that directory already exists a fresh
# TAG_2, TAG_3, ... is used, so a re-run never overwrites a failing log.  Every
# GPU step runs under its own time limit; the script stops at the first step
# that faults / aborts / times out (rc other than 0 or 1) and, for the test
# steps, at a failing test too (rc 1).  Extra bench.py flags for the bench
# steps: BENCH_ARGS="--steps 5"; an A/B library: SMJ_LIB=/path/libsmj_hip.so.
set -u
TAG=${1:-run}; shift || true
STEPS=${*:-smoke tests c3 prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
i=2
while [ -e "$OUT" ]; do OUT=$ROOT/gpurun_out/${TAG}_$i; i=$((i + 1)); done
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
# the library's source hash on the box: PMC summaries are keyed by it (tools/pmc_traffic.py)
python3 -c "import sys; sys.path.insert(0, 'pim-sort-merge-join_amd'); from smj._lib import source_sha; print(source_sha())" > "$OUT/source_sha.txt" 2>/dev/null || true
BA=${BENCH_ARGS:-}
NOCPU="--cpu-sample 0 --cpu-mt 0"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
run() {  # name timeout cmd...   (rc 1 tolerated: a bench step's stderr is read afterwards)
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" | tee -a "$OUT/steps.log"; exit $rc; fi
  # a GPU fault inside a Python step surfaces as an exception (rc 1): stop there too
  if [ $rc -ne 0 ] && grep -qE "HSA_STATUS_ERROR|Memory access fault|hardware exception|unspecified launch failure|hipErrorLaunchFailure|page not present|illegal memory access" "$OUT/$name.err"; then
    echo "stopping after $name (GPU fault in stderr)" | tee -a "$OUT/steps.log"; exit 3
  fi
  return $rc
}
test_run() {  # a pytest step: stop on any failure
  run "$@" || { tail -30 "$OUT/$1.out"; echo "stopping after $1 (tests failed)" | tee -a "$OUT/steps.log"; exit 1; }
}
summ() {  # one-line summary of a bench JSON
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], d['ms_per_step'], 'ms/step', d['value'], 'verified', d.get('verified'), r.get('kernel'), r.get('frac'), {k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 0.1})" "$1" "$2" | tee -a "$OUT/steps.log"
}
for s in $STEPS; do
  case $s in
    smoke) test_run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) test_run tests 1200 $PYT tests -m gpu ;;
    msd)   test_run msd 600 $PYT tests/test_gpu_msd.py ;;
    parity) test_run parity 600 $PYT tests/test_gpu_parity.py ;;
    large) test_run large 900 $PYT tests/test_gpu_large.py ;;
    lsmall) test_run lsmall 600 $PYT tests/test_gpu_large.py -k "partition or chunked" ;;
    lfull) test_run lfull 900 $PYT tests/test_gpu_large.py -k "full_size" ;;
    dist)  test_run dist 600 $PYT tests/test_dist_gloo.py -m gpu ;;
    multidev) test_run multidev 600 $PYT tests/test_gpu_multidev.py ;;
    benchtest) test_run benchtest 600 $PYT tests/test_gpu_bench.py ;;
    pkt)   test_run pkt 600 $PYT tests/test_gpu_msd.py -k packed_pass_b ;;
    msdpk2) SMJ_PACKB=2 test_run msdpk2 600 $PYT tests/test_gpu_msd.py ;;
    msdpk0) SMJ_PACKB=0 test_run msdpk0 600 $PYT tests/test_gpu_msd.py ;;
    largepk2) SMJ_PACKB=2 test_run largepk2 900 $PYT tests/test_gpu_large.py ;;
    largeh) SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/headv/libsmj_hip.so test_run largeh 900 $PYT tests/test_gpu_large.py ;;
    c3)    run c3 400 python bench.py $BA && summ "$OUT/c3.out" c3 ;;
    quick) run quick 300 python bench.py $NOCPU $BA && summ "$OUT/quick.out" c3 ;;
    krange) for k in 300000000 1000000000 2147483648 4000000000 8000000000 30000000000 1000000000000; do
              run kr$k 300 python bench.py --key-range $k $NOCPU && summ "$OUT/kr$k.out" c3_keyrange_$k
            done ;;
    c3w)   run c3w 400 python bench.py --workload c3w $NOCPU $BA && summ "$OUT/c3w.out" c3w ;;
    c3wv)  run c3wv 600 python bench.py --workload c3w $BA && summ "$OUT/c3wv.out" c3w ;;
    c3w7)  run c3w7 300 python bench.py --workload c3w --rows 10000000 $NOCPU $BA && summ "$OUT/c3w7.out" c3w_1e7 ;;
    c4v)   run c4v 900 python bench.py --workload c4 --steps 5 --warmup 2 --cpu-sample 0 $BA && summ "$OUT/c4v.out" c4 ;;
    c5v)   run c5v 900 python bench.py --workload c5 --steps 5 --warmup 2 --cpu-sample 0 $BA && summ "$OUT/c5v.out" c5 ;;
    c4)    run c4 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU $BA && summ "$OUT/c4.out" c4 ;;
    c5)    run c5 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU $BA && summ "$OUT/c5.out" c5 ;;
    c4old) SMJ_PART1C=0 run c4old 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU $BA && summ "$OUT/c4old.out" c4old ;;
    c4pf)  SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/p1cpf/libsmj_hip.so run c4pf 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU $BA && summ "$OUT/c4pf.out" c4pf ;;
    c4nov) SMJ_PART_OVERLAP=0 run c4nov 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU $BA && summ "$OUT/c4nov.out" c4nov ;;
    c5nov) SMJ_PART_OVERLAP=0 run c5nov 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU $BA && summ "$OUT/c5nov.out" c5nov ;;
    hostc4) SMJ_DEBUG_HOST=1 run hostc4 600 python bench.py --workload c4 --steps 3 --warmup 1 $NOCPU ;;
    hostc5) SMJ_DEBUG_HOST=1 run hostc5 600 python bench.py --workload c5 --steps 3 --warmup 1 $NOCPU ;;
    abov)  # same-box A/B/C of the partitioned mode's part overlap: on / chained / off, twice, C4 and C5
           for w in c4 c5; do for r in 1 2; do
             run ab_${w}_on_$r 600 python bench.py --workload $w --steps 5 --warmup 2 $NOCPU && summ "$OUT/ab_${w}_on_$r.out" ${w}_on
             SMJ_PART_CHAIN=1 run ab_${w}_ch_$r 600 python bench.py --workload $w --steps 5 --warmup 2 $NOCPU && summ "$OUT/ab_${w}_ch_$r.out" ${w}_chain
             SMJ_PART_OVERLAP=0 run ab_${w}_off_$r 600 python bench.py --workload $w --steps 5 --warmup 2 $NOCPU && summ "$OUT/ab_${w}_off_$r.out" ${w}_off
           done; done ;;
    abparts) for r in 1 2 3 4; do
             run pr7_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/pr7_$r.out" c4_p7
             SMJ_PART_ROWS=72000000 run pr14_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/pr14_$r.out" c4_p14
           done ;;
    abparts2) for r in 1 2; do
             for pr in 72000000 50000000 36000000; do
               SMJ_PART_ROWS=$pr run c4r${pr}_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4r${pr}_$r.out" c4_rows$pr
             done
             for pr in 150000000 100000000; do
               SMJ_PART_ROWS=$pr run c5r${pr}_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5r${pr}_$r.out" c5_rows$pr
             done
           done ;;
    c5knobs) for r in 1 2; do
             for pr in 80000000 100000000 125000000; do
               SMJ_PART_ROWS=$pr run c5p${pr}_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5p${pr}_$r.out" c5_rows$pr
             done
             SMJ_BG_SEG=16384 run c5seg16k_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5seg16k_$r.out" c5_seg16k
             SMJ_BG_MAX_ROWS=32768 run c5bg32k_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5bg32k_$r.out" c5_bgmax32k
           done ;;
    loopk) for r in 1 2; do
             for k in ${LOOPK:-2 3 4}; do
               SMJ_DIST_STAGES=$k run loopk${k}_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/loopk${k}_$r.out" loop_k$k
             done
           done ;;
    abpa)  for r in 1 2 3; do
             run c3pa0_$r 300 python bench.py $NOCPU && summ "$OUT/c3pa0_$r.out" c3_pa_tile
             SMJ_PA_PERSIST=1 run c3pa1_$r 300 python bench.py $NOCPU && summ "$OUT/c3pa1_$r.out" c3_pa_persist
           done
           for r in 1 2; do
             run c4pa0_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4pa0_$r.out" c4_pa_tile
             SMJ_PA_PERSIST=1 run c4pa1_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4pa1_$r.out" c4_pa_persist
           done ;;
    abp1i) V=$ROOT/pim-sort-merge-join_amd/lib/variants
           for r in 1 2; do
             run c4i8_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4i8_$r.out" c4_p1items8
             SMJ_LIB=$V/p1i4/libsmj_hip.so run c4i4_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4i4_$r.out" c4_p1items4
             SMJ_LIB=$V/p1i6/libsmj_hip.so run c4i6_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4i6_$r.out" c4_p1items6
           done ;;
    abp1l) V=$ROOT/pim-sort-merge-join_amd/lib/variants  # same-box A/B of the partition tile on the loopback C3 line
           for r in 1 2; do
             run lp8_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/lp8_$r.out" loop_p1items8
             for i in 4 6 12; do
               SMJ_LIB=$V/p1i$i/libsmj_hip.so run lp${i}_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/lp${i}_$r.out" loop_p1items$i
             done
           done ;;
    abp1pk) V=$ROOT/pim-sort-merge-join_amd/lib/variants  # same-box A/B of the packed-staging partition (loopback C3)
           for r in 1 2; do
             SMJ_LIB=$V/p1head/libsmj_hip.so run lph_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/lph_$r.out" loop_head
             run lpk4_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/lpk4_$r.out" loop_pk_wpe4
             for i in 6 8; do
               SMJ_LIB=$V/p1pk$i/libsmj_hip.so run lpk${i}_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/lpk${i}_$r.out" loop_pk_wpe$i
             done
           done ;;
    abpkb) for r in 1 2; do  # same-box A/B of packed pass-B rows (SMJ_PACKB)
             run c3pk1_$r 300 python bench.py $NOCPU && summ "$OUT/c3pk1_$r.out" c3_packb
             SMJ_PACKB=0 run c3pk0_$r 300 python bench.py $NOCPU && summ "$OUT/c3pk0_$r.out" c3_rows
           done
           for r in 1 2; do
             run c4pk1_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4pk1_$r.out" c4_packb
             SMJ_PACKB=0 run c4pk0_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4pk0_$r.out" c4_rows
             run c5pk1_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5pk1_$r.out" c5_packb
             SMJ_PACKB=0 run c5pk0_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5pk0_$r.out" c5_rows
           done ;;
    abpkr) V=$ROOT/pim-sort-merge-join_amd/lib/variants  # packed pass-B rows: runtime-branch kernels vs dual launches vs rows
           for r in 1 2; do
             run c3r_$r 300 python bench.py $NOCPU && summ "$OUT/c3r_$r.out" c3_pk_runtime
             SMJ_LIB=$V/pkdual/libsmj_hip.so run c3d_$r 300 python bench.py $NOCPU && summ "$OUT/c3d_$r.out" c3_pk_dual
             SMJ_PACKB=0 run c3o_$r 300 python bench.py $NOCPU && summ "$OUT/c3o_$r.out" c3_rows
           done
           for r in 1 2; do
             run c4r_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4r_$r.out" c4_pk_runtime
             SMJ_PACKB=0 run c4o_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4o_$r.out" c4_rows
             run c5r_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5r_$r.out" c5_pk_runtime
             SMJ_PACKB=0 run c5o_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5o_$r.out" c5_rows
           done ;;
    abpka) for r in 1 2; do  # same-box A/B of packed pass-A tiles (SMJ_PACKA)
             run c3a1_$r 300 python bench.py $NOCPU && summ "$OUT/c3a1_$r.out" c3_packa
             SMJ_PACKA=0 run c3a0_$r 300 python bench.py $NOCPU && summ "$OUT/c3a0_$r.out" c3_rowsa
           done
           for r in 1 2; do
             run c4a1_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4a1_$r.out" c4_packa
             SMJ_PACKA=0 run c4a0_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4a0_$r.out" c4_rowsa
             run c5a1_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5a1_$r.out" c5_packa
             SMJ_PACKA=0 run c5a0_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5a0_$r.out" c5_rowsa
           done ;;
    ab:*)  # ab:VARIANT -- same-box A/B of lib/variants/VARIANT against lib/variants/headv: C3 x3, C3-wide x2
           V=$ROOT/pim-sort-merge-join_amd/lib/variants; vn=${s#ab:}
           for r in 1 2 3; do
             SMJ_LIB=$V/$vn/libsmj_hip.so run c3${vn}_$r 300 python bench.py $NOCPU && summ "$OUT/c3${vn}_$r.out" c3_$vn
             SMJ_LIB=$V/headv/libsmj_hip.so run c3h_$r 300 python bench.py $NOCPU && summ "$OUT/c3h_$r.out" c3_head
           done
           for r in 1 2; do
             SMJ_LIB=$V/$vn/libsmj_hip.so run c3w${vn}_$r 300 python bench.py --workload c3w $NOCPU && summ "$OUT/c3w${vn}_$r.out" c3w_$vn
             SMJ_LIB=$V/headv/libsmj_hip.so run c3wh_$r 300 python bench.py --workload c3w $NOCPU && summ "$OUT/c3wh_$r.out" c3w_head
           done ;;
    ab4:*) # ab4:VARIANT -- same-box A/B on C4 (two rounds) and C5 (one)
           V=$ROOT/pim-sort-merge-join_amd/lib/variants; vn=${s#ab4:}
           for r in 1 2; do
             SMJ_LIB=$V/$vn/libsmj_hip.so run c4${vn}_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4${vn}_$r.out" c4_$vn
             SMJ_LIB=$V/headv/libsmj_hip.so run c4h_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4h_$r.out" c4_head
           done
           SMJ_LIB=$V/$vn/libsmj_hip.so run c5${vn} 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5${vn}.out" c5_$vn
           SMJ_LIB=$V/headv/libsmj_hip.so run c5h 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5h.out" c5_head ;;
    abhv)  V=$ROOT/pim-sort-merge-join_amd/lib/variants  # working tree vs the HEAD build (headv), C3, three rounds
           for r in 1 2 3; do
             run c3n_$r 300 python bench.py $NOCPU && summ "$OUT/c3n_$r.out" c3_new
             SMJ_LIB=$V/headv/libsmj_hip.so run c3h_$r 300 python bench.py $NOCPU && summ "$OUT/c3h_$r.out" c3_head
           done ;;
    abst)  V=$ROOT/pim-sort-merge-join_amd/lib/variants  # staged-kernel grid / record-ring variants, C3
           for r in 1 2 3; do
             run st0_$r 300 python bench.py $NOCPU && summ "$OUT/st0_$r.out" c3_grid768
             for n in stg1024 stg1536 strec8; do
               SMJ_LIB=$V/$n/libsmj_hip.so run ${n}_$r 300 python bench.py $NOCPU && summ "$OUT/${n}_$r.out" c3_$n
             done
           done ;;
    abdef) V=$ROOT/pim-sort-merge-join_amd/lib/variants  # deferred packed-word decode vs HEAD (headv); C4 with packed parts too
           for r in 1 2 3; do
             run c3n_$r 300 python bench.py $NOCPU && summ "$OUT/c3n_$r.out" c3_new
             SMJ_LIB=$V/headv/libsmj_hip.so run c3h_$r 300 python bench.py $NOCPU && summ "$OUT/c3h_$r.out" c3_head
           done
           for r in 1 2; do
             SMJ_PACKB=2 run c4n2_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4n2_$r.out" c4_new_packedparts
             run c4n_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4n_$r.out" c4_new
           done ;;
    abc5l) for r in 1 2; do  # C5 and the loopback line: packed pass-B rows allowed (default) vs off
             run c5d_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5d_$r.out" c5_default
             SMJ_PACKB=0 run c5o_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5o_$r.out" c5_packb0
             run lpd_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/lpd_$r.out" loop_default
             SMJ_PACKB=0 run lpo_$r 300 python bench.py --loopback $NOCPU && summ "$OUT/lpo_$r.out" loop_packb0
           done ;;
    abearly) V=$ROOT/pim-sort-merge-join_amd/lib/variants  # equal-key rounds: early exit (default) vs all fl rounds
           for r in 1 2 3; do
             run c3e_$r 300 python bench.py $NOCPU && summ "$OUT/c3e_$r.out" c3_early
             SMJ_LIB=$V/noearly/libsmj_hip.so run c3f_$r 300 python bench.py $NOCPU && summ "$OUT/c3f_$r.out" c3_allrounds
           done
           run c5e 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5e.out" c5_early
           SMJ_LIB=$V/noearly/libsmj_hip.so run c5f 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5f.out" c5_allrounds ;;
    abei)  V=$ROOT/pim-sort-merge-join_amd/lib/variants  # early issue of the next group's gathers vs HEAD (headv)
           for r in 1 2 3; do
             run c3n_$r 300 python bench.py $NOCPU && summ "$OUT/c3n_$r.out" c3_new
             SMJ_LIB=$V/headv/libsmj_hip.so run c3h_$r 300 python bench.py $NOCPU && summ "$OUT/c3h_$r.out" c3_head
           done
           for r in 1 2; do
             run c4n_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4n_$r.out" c4_new
             SMJ_LIB=$V/headv/libsmj_hip.so run c4h_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4h_$r.out" c4_head
           done ;;
    abph)  V=$ROOT/pim-sort-merge-join_amd/lib/variants  # packed pass-B rows with heavy keys (C5) vs HEAD (headv)
           for r in 1 2; do
             run c5n_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5n_$r.out" c5_new
             SMJ_LIB=$V/headv/libsmj_hip.so run c5h_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5h_$r.out" c5_head
           done
           run c3n 300 python bench.py $NOCPU && summ "$OUT/c3n.out" c3_new
           SMJ_LIB=$V/headv/libsmj_hip.so run c3h 300 python bench.py $NOCPU && summ "$OUT/c3h.out" c3_head ;;
    abph2) V=$ROOT/pim-sort-merge-join_amd/lib/variants  # working tree vs HEAD (headv): C3 x3, C5 x2
           for r in 1 2 3; do
             run c3n_$r 300 python bench.py $NOCPU && summ "$OUT/c3n_$r.out" c3_new
             SMJ_LIB=$V/headv/libsmj_hip.so run c3h_$r 300 python bench.py $NOCPU && summ "$OUT/c3h_$r.out" c3_head
           done
           for r in 1 2; do
             run c5n_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5n_$r.out" c5_new
             SMJ_LIB=$V/headv/libsmj_hip.so run c5h_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5h_$r.out" c5_head
           done ;;
    abbase) V=$ROOT/pim-sort-merge-join_amd/lib/variants/base/libsmj_hip.so
           for r in 1 2 3; do
             run c3new_$r 300 python bench.py $NOCPU && summ "$OUT/c3new_$r.out" c3_new
             SMJ_LIB=$V run c3base_$r 300 python bench.py $NOCPU && summ "$OUT/c3base_$r.out" c3_base
           done
           for r in 1 2; do
             run c4new_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4new_$r.out" c4_new
             SMJ_LIB=$V run c4base_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4base_$r.out" c4_base
           done ;;
    abpbo) for r in 1 2 3; do
             run c3o1_$r 300 python bench.py $NOCPU && summ "$OUT/c3o1_$r.out" c3_order
             SMJ_PB_ORDER=0 run c3o0_$r 300 python bench.py $NOCPU && summ "$OUT/c3o0_$r.out" c3_plain
           done
           for r in 1 2; do
             run c4o1_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4o1_$r.out" c4_order
             SMJ_PB_ORDER=0 run c4o0_$r 600 python bench.py --workload c4 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c4o0_$r.out" c4_plain
           done ;;
    loop)  run loop 300 python bench.py --loopback $NOCPU $BA && summ "$OUT/loop.out" loop ;;
    loopnp) SMJ_DIST_PACK=0 run loopnp 300 python bench.py --loopback $NOCPU $BA && summ "$OUT/loopnp.out" loop_nopack ;;
    loopns) SMJ_DIST_SPLIT=0 run loopns 300 python bench.py --loopback $NOCPU $BA && summ "$OUT/loopns.out" loop_nosplit ;;
    loopab) for r in 1 2 3; do
              run loop_s$r 300 python bench.py --loopback $NOCPU $BA && summ "$OUT/loop_s$r.out" loop_split
              SMJ_DIST_SPLIT=0 run loop_n$r 300 python bench.py --loopback $NOCPU $BA && summ "$OUT/loop_n$r.out" loop_nosplit
            done ;;
    trl4)  run trl4 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trl4" -o l4 -- \
               python3 "$ROOT/bench.py" --loopback --workload c4 --steps 2 --warmup 1 $NOCPU --verify 0 ;;
    loop4tr) SMJ_DIST_TRACE=2 run loop4tr 900 python bench.py --loopback --workload c4 --steps 3 --warmup 1 $NOCPU $BA && summ "$OUT/loop4tr.out" loop_c4_trace ;;
    memwait) # until the previous step's process has its device memory back (r06y5: a loopback C4 right
             # after another large run waited 0.5 s in its exchange allocation)
             python3 -c "
import sys, time, torch
t0 = time.time()
while True:
    free, total = torch.cuda.mem_get_info()
    if total - free < 8 * 2 ** 30 or time.time() - t0 > 180:
        print('memwait %.1f s, %.1f GiB held' % (time.time() - t0, (total - free) / 2 ** 30)); break
    time.sleep(0.5)
" | tee -a "$OUT/steps.log" ;;
    loop4s0) SMJ_SEG=0 run loop4s0 900 python bench.py --loopback --workload c4 --steps 3 --warmup 1 $NOCPU $BA && summ "$OUT/loop4s0.out" loop_c4_seg0 ;;
    loop4) run loop4 900 python bench.py --loopback --workload c4 --steps 3 --warmup 1 $NOCPU $BA && summ "$OUT/loop4.out" loop_c4 ;;
    loop5) run loop5 900 python bench.py --loopback --workload c5 --steps 3 --warmup 1 $NOCPU $BA && summ "$OUT/loop5.out" loop_c5 ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c3 -- \
               python3 "$ROOT/bench.py" --steps 10 --warmup 2 $NOCPU
           rm -f "$OUT/prof/c3_kernel_trace.csv" ;;
    prof4pk) for m in 2 1; do  # C4 kernel stats with the parts' pass-B rows packed (2) / not (1)
               SMJ_PACKB=$m run prof4pk$m 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof4pk$m" -o c4 -- \
                 python3 "$ROOT/bench.py" --workload c4 --steps 3 --warmup 1 $NOCPU
               rm -f "$OUT/prof4pk$m/c4_kernel_trace.csv"
             done ;;
    prof5) run prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5" -o c5 -- \
               python3 "$ROOT/bench.py" --workload c5 --steps 2 --warmup 1 $NOCPU
           rm -f "$OUT/prof5/c5_kernel_trace.csv" ;;
    prof4) run prof4 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof4" -o c4 -- \
               python3 "$ROOT/bench.py" --workload c4 --steps 2 --warmup 1 $NOCPU
           rm -f "$OUT/prof4/c4_kernel_trace.csv" ;;
    prof5n|prof5n0)  # C5 kernel stats with the parts serialised (no overlap), heavy keys on / off
           h=1; [ $s = prof5n0 ] && h=0
           SMJ_HEAVY=$h SMJ_PART_OVERLAP=0 run $s 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$s" -o c5 -- \
               python3 "$ROOT/bench.py" --workload c5 --steps 2 --warmup 1 $NOCPU
           rm -f "$OUT/$s/c5_kernel_trace.csv" ;;
    proflp) run proflp 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/proflp" -o loop -- \
               python3 "$ROOT/bench.py" --loopback --steps 5 --warmup 2 $NOCPU
           rm -f "$OUT/proflp/loop_kernel_trace.csv" ;;
    tr5)   run tr5 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr5" -o c5 -- \
               python3 "$ROOT/bench.py" --workload c5 --steps 2 --warmup 1 $NOCPU
           python3 tools/trace_gaps.py "$OUT/tr5/c5_kernel_trace.csv" --from-kernel msd_sample --top 30 --per msd_part_sample > "$OUT/tr5_gaps.txt" ;;
    tr4)   run tr4 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr4" -o c4 -- \
               python3 "$ROOT/bench.py" --workload c4 --steps 2 --warmup 1 $NOCPU
           python3 tools/trace_gaps.py "$OUT/tr4/c4_kernel_trace.csv" --from-kernel msd_sample --top 30 --per msd_part_sample > "$OUT/tr4_gaps.txt" ;;
    trlp)  run trlp 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trlp" -o loop -- \
               python3 "$ROOT/bench.py" --loopback --steps 3 --warmup 1 $NOCPU
           python3 tools/trace_gaps.py "$OUT/trlp/loop_kernel_trace.csv" --from-kernel msd_sample --top 30 --per p1_set_words > "$OUT/trlp_gaps.txt" ;;
    p1)    run p1_base 300 python tools/p1_probe.py && \
           SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/p1abl/libsmj_hip.so run p1_abl 300 python tools/p1_probe.py ;;
    pmcf)  run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
               python3 "$ROOT/bench.py" --steps 2 --warmup 1 $NOCPU $BA ;;
    pmcw)  run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
               python3 "$ROOT/bench.py" --steps 2 --warmup 1 $NOCPU $BA ;;
    pmc45) for w in c4 c5; do
             run pmc_fetch_$w 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$w" -o run -- \
               python3 "$ROOT/bench.py" --workload $w --steps 2 --warmup 1 $NOCPU
             run pmc_write_$w 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$w" -o run -- \
               python3 "$ROOT/bench.py" --workload $w --steps 2 --warmup 1 $NOCPU
           done ;;
    pmc:*) # pmc:WORKLOAD -- FETCH_SIZE and WRITE_SIZE passes (separate runs) of bench.py --workload WORKLOAD
           w=${s#pmc:}; st="--steps 2 --warmup 1"; [ "$w" = c4 ] || [ "$w" = c5 ] && st="--steps 1 --warmup 1"
           run pmc_fetch_$w 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$w" -o run -- \
               python3 "$ROOT/bench.py" --workload $w $st $NOCPU --verify 0 && \
           run pmc_write_$w 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$w" -o run -- \
               python3 "$ROOT/bench.py" --workload $w $st $NOCPU --verify 0 ;;
    kstat:*) # kstat:WORKLOAD -- rocprofv3 kernel stats of bench.py --workload WORKLOAD
           w=${s#kstat:}
           run kstat_$w 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstat_$w" -o $w -- \
               python3 "$ROOT/bench.py" --workload $w --steps 10 --warmup 2 $NOCPU --verify 0
           rm -f "$OUT/kstat_$w/${w}_kernel_trace.csv" ;;
    pmcsq) run pmc_sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
               --output-format csv -d "$OUT/pmc_sq" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 $NOCPU $BA ;;
    pmcsq2) run pmc_sq2 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES \
               --output-format csv -d "$OUT/pmc_sq2" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 $NOCPU $BA ;;
    pmclist) run pmclist 60 rocprofv3 -L ;;
    shapes) run shapes 600 python tools/shape_probe.py ;;
    shapesh) SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/headv/libsmj_hip.so run shapesh 600 python tools/shape_probe.py ;;
    seg)   test_run seg 600 $PYT tests/test_gpu_msd.py -k clustered ;;
    lsdt)  test_run lsdt 600 $PYT tests/test_gpu_msd.py -k "single_key_groups_skip or long_equal_key or zipf or heavy" ;;
    sortt) test_run sortt 600 $PYT tests/test_gpu_msd.py -k "sorted_input" ;;
    segp)  run segp 600 python tools/seg_probe.py ;;
    segst) test_run segst 600 python -u tools/seg_stress.py 0 400 420 ;;
    segst2) test_run segst2 600 python -u tools/seg_stress.py 400 1600 420 ;;
    segmix) test_run segmix 600 python -u tools/seg_stress.py --mixed 0 400 420 ;;
    seghost) test_run seghost 600 python -u tools/seg_stress.py --host 0 300 420 ;;
    segmix2) test_run segmix2 600 python -u tools/seg_stress.py --mixed 400 1200 420 ;;
    segtyped) test_run segtyped 600 python -u tools/seg_stress.py --typed 0 400 420 ;;
    seghostbig) test_run seghostbig 600 python -u tools/seg_stress.py --hostbig 0 60 400 ;;
    bigst) run bigst 600 python -u tools/big_stress.py ;;
    extp)  run extp 300 python -u tools/ext_probe.py ${EXTP_SEEDS:-25 29 38 86} ;;
    segd)  SD=--seeds=${SEGD_SEEDS:-11,25,29,38,86,146,399}  # failing stress seeds in detail, under each switch
           run segd_def 300 python -u tools/seg_stress.py $SD
           SMJ_SEG=0 run segd_noseg 300 python -u tools/seg_stress.py $SD
           SMJ_ST_COMBINED=0 run segd_comb0 300 python -u tools/seg_stress.py $SD
           SMJ_ST_COMBINED=1 run segd_comb1 300 python -u tools/seg_stress.py $SD
           SMJ_PACKB=0 run segd_pk0 300 python -u tools/seg_stress.py $SD
           SMJ_HEAVY=0 run segd_hv0 300 python -u tools/seg_stress.py $SD ;;
    kbis)  V=$ROOT/pim-sort-merge-join_amd/lib/variants  # bases-kernel bisection: kernel stats per variant
           for v in bis1 headv; do
             SMJ_LIB=$V/$v/libsmj_hip.so run kstat_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstat_$v" -o c3 -- \
               python bench.py --workload c3 --steps 5 --warmup 2 $NOCPU || exit 1
             rm -f "$OUT/kstat_$v/c3_kernel_trace.csv"
           done ;;
    phases) run phases 300 python tools/msd_phases.py ;;
    finab) run finab 300 python tools/final_ablate.py ;;
    finabv) SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/ablate/libsmj_hip.so run finabv 300 python tools/final_ablate.py ;;
    finv)  V=$ROOT/pim-sort-merge-join_amd/lib/variants  # phases (stamps build) + ablation (ablate build) on HEAD
           SMJ_LIB=$V/stamps/libsmj_hip.so run phasesv 300 python tools/msd_phases.py && \
           SMJ_LIB=$V/ablate/libsmj_hip.so run finabv 300 python tools/final_ablate.py ;;
    pbab)  run pbab 300 python tools/pb_ablate.py ;;
    t:*)   # t:FILE[:KEXPR] -- one test file, optionally filtered by -k (underscores kept, '+' = space)
           spec=${s#t:}; f=${spec%%:*}; k=""; [ "$spec" != "$f" ] && k=${spec#*:}
           n=$(basename "$f" .py)_$(echo "$k" | tr -c 'a-zA-Z0-9' '_' | cut -c1-30)
           if [ -n "$k" ]; then test_run "$n" 1200 $PYT "$f" -m gpu -k "${k//+/ }"
           else test_run "$n" 1200 $PYT "$f" -m gpu; fi ;;
    dbg3)  SMJ_DIST_TRACE=1 run dbg3 170 python -u bench.py --loopback --steps 3 --warmup 1 $NOCPU ;;
    dbg4)  SMJ_DIST_TRACE=1 SMJ_DEBUG_PART1=1 run dbg4 170 python -u bench.py --loopback --workload c4 --steps 1 --warmup 0 $NOCPU ;;
    dbg4s) SMJ_DIST_TRACE=2 SMJ_DEBUG_PART1=1 SMJ_DEBUG_HOST=1 run dbg4s 170 python -u bench.py --loopback --workload c4 --steps 2 --warmup 1 $NOCPU ;;
    dbg4h0) SMJ_HEAVY=0 SMJ_DEBUG_PART1=1 SMJ_DEBUG_HOST=1 run dbg4h0 170 python -u bench.py --loopback --workload c4 --steps 2 --warmup 1 $NOCPU ;;
    seqb)  SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/bounds/libsmj_hip.so SMJ_DEBUG_PART1=1 SMJ_DEBUG_HOST=1 run seqb 170 python -u tools/seq_sizes.py ;;
    sb:*)  # sb:SEQ -- the size-sequence probe on the bounds-checking build (reports instead of faulting)
           q=${s#sb:}; SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/bounds/libsmj_hip.so SMJ_DEBUG_PART1=1 run sb_$(echo $q | tr -c 'a-z0-9' '_') 170 python -u tools/seq_sizes.py --seq $q ;;
    sr4:*) # sr4:SEQ -- the same probe on round 4's library (db75936) built with the bounds checks
           q=${s#sr4:}; SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/r4b/libsmj_hip.so SMJ_DEBUG_PART1=1 run sr4_$(echo $q | tr -c 'a-z0-9' '_') 170 python -u tools/seq_sizes.py --seq $q ;;
    sv:*)  # sv:VARIANT:SEQ -- the probe on lib/variants/VARIANT
           r=${s#sv:}; v=${r%%:*}; q=${r#*:}; SMJ_LIB=$ROOT/pim-sort-merge-join_amd/lib/variants/$v/libsmj_hip.so SMJ_DEBUG_PART1=1 run sv_${v}_$(echo $q | tr -c 'a-z0-9' '_') 170 python -u tools/seq_sizes.py --seq $q ;;
    seq)   SMJ_DEBUG_PART1=1 SMJ_DEBUG_HOST=1 run seq 170 python -u tools/seq_sizes.py ;;
    dbg4n) SMJ_DIST_S_SIDE=0 SMJ_DIST_TRACE=1 SMJ_DEBUG_PART1=1 run dbg4n 170 python -u bench.py --loopback --workload c4 --steps 1 --warmup 0 $NOCPU ;;
    abpk)  for r in 1 2; do  # same-box A/B of packed parts in the partitioned mode, C4 and C5
             for w in c4 c5; do
               run ${w}pk1_$r 600 python bench.py --workload $w --steps 5 --warmup 2 $NOCPU && summ "$OUT/${w}pk1_$r.out" ${w}_packed
               SMJ_PART_PACK=0 run ${w}pk0_$r 600 python bench.py --workload $w --steps 5 --warmup 2 $NOCPU && summ "$OUT/${w}pk0_$r.out" ${w}_plain
             done
           done ;;
    abh5)  for r in 1 2; do  # same-box A/B of heavy-key sub-buckets on C5
             run c5h1_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5h1_$r.out" c5_heavy
             SMJ_HEAVY=0 run c5h0_$r 600 python bench.py --workload c5 --steps 5 --warmup 2 $NOCPU && summ "$OUT/c5h0_$r.out" c5_noheavy
           done ;;
    loopv) for w in c3 c4 c5; do
             run loopv_$w 900 python bench.py --loopback --workload $w --steps 3 --warmup 1 $NOCPU $BA && summ "$OUT/loopv_$w.out" loop_$w
           done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done ($OUT)" | tee -a "$OUT/steps.log"
