# staged final kernel phase stamps (SMJ_STAMPS build): C3 and C5
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
L=pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so
SMJ_LIB=$L timeout -k 10 300 python tools/msd_phases.py > $O/c3_phases.txt 2> $O/c3_phases.err || { echo "c3 rc=$?"; tail -5 $O/c3_phases.err; exit 1; }
cat $O/c3_phases.txt
SMJ_LIB=$L WORKLOAD=c5 timeout -k 10 300 python tools/msd_phases.py > $O/c5_phases.txt 2> $O/c5_phases.err || { echo "c5 rc=$?"; tail -5 $O/c5_phases.err; exit 1; }
cat $O/c5_phases.txt
