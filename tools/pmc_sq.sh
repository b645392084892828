#!/bin/bash
# tools/pmc_sq.sh TAG -- two SQ counter passes over the C3 bench (dynamic
# instruction mix and wave-cycle breakdown per kernel), each its own run
# under a hard limit; summarise with tools/pmc_sq_sum.py TAG.
set -o pipefail
TAG=$1; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; O=$ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B="python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 --cpu-mt 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH \
    --output-format csv -d $O/sq1 -o run -- $B > $O/sq1.out 2> $O/sq1.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_LDS_ATOMIC SQ_WAIT_INST_LDS \
    --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.out 2> $O/sq2.err
