# C5 group statistics (one part) and C5 phase stamps of the staged final kernel
set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/c5_groups.py > $O/c5_groups.json 2> $O/c5_groups.err || { echo "groups rc=$?"; tail -5 $O/c5_groups.err; exit 1; }
cat $O/c5_groups.json
WORKLOAD=c5 SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so timeout -k 10 300 python tools/msd_phases.py > $O/c5_phases.txt 2>&1 || { echo "phases rc=$?"; tail -5 $O/c5_phases.txt; exit 1; }
cat $O/c5_phases.txt
