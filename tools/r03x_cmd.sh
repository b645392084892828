# C5 oversized-group sizes (combined groups) and big-group phase cycles
set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
export TMPDIR=/tmp
SMJ_DEBUG_BIG=1 timeout -k 10 300 python tools/c5_groups.py > $O/c5_groups.json 2> $O/c5_big_sizes.txt || { echo "groups rc=$?"; tail -5 $O/c5_big_sizes.txt; exit 1; }
cat $O/c5_groups.json; grep "big groups" $O/c5_big_sizes.txt | tail -40
SMJ_LIB=$PWD/pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so SMJ_DEBUG_BIG=1 timeout -k 10 300 python tools/big_times.py > $O/big_times.json 2> $O/big_times.err || { echo "big rc=$?"; tail -5 $O/big_times.err; exit 1; }
cat $O/big_times.json
