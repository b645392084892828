#!/bin/bash
# tools/gpu_run.sh TAG [steps...] -- the standard GPU-box sequence.  Every
# GPU step runs under its own time limit; the script stops at the first
# step that faults / aborts / times out (rc other than 0 or 1).
# Steps: smoke tests bench prof pmc (default: smoke tests bench prof)
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-smoke tests bench prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() {  # name timeout cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" | tee -a "$OUT/steps.log"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    build) run build 600 make -s -j16 -C pim-sort-merge-join_amd ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    msd)   run msd 600 python -u -m pytest tests/test_gpu_msd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    dist)  run dist 600 python -u -m pytest tests/test_dist_gloo.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    quick) run quick 300 python bench.py --cpu-sample 0 --cpu-mt 0 ;;
    qfull) SMJ_PASSB_FULL=1 run qfull 300 python bench.py --cpu-sample 0 --cpu-mt 0 ;;
    phases) run phases 300 python tools/msd_phases.py ;;
    l3)    run l3 300 python tools/l3_probe.py ;;
    large) run large 900 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider ;;
    pbab)  run pbab 300 python tools/pb_ablate.py ;;
    finab) run finab 300 python tools/final_ablate.py ;;
    h2d)   run h2d 300 python tools/h2d_probe.py ;;
    part)  run part 300 python tools/part_probe.py ;;
    ptest) run ptest 600 python -u -m pytest tests -m gpu -x -v -k "partition or distributed" --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    typed) run typed 600 python -u -m pytest tests -m gpu -x -q -k "typed" --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    prof)  export TMPDIR=/tmp
           run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
               python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --cpu-mt 0
           rm -f "$OUT/prof/run_kernel_trace.csv" ;;
    pmcf)  export TMPDIR=/tmp
           run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
               python "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 ;;
    pmcsq) export TMPDIR=/tmp
           run pmc_sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS \
               --output-format csv -d "$OUT/pmc_sq" -o run -- python "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 ;;
    pmcw)  export TMPDIR=/tmp
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
               python "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done" | tee -a "$OUT/steps.log"
