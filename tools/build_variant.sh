#!/bin/bash
# tools/build_variant.sh NAME "-DFLAG=.. ..." -- build libsmj_hip.so with extra
# compile flags into pim-sort-merge-join_amd/lib/variants/NAME/ (A/B runs load
# it through SMJ_LIB=...).
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../pim-sort-merge-join_amd"
OUT=lib/variants/$NAME; mkdir -p $OUT build/v_$NAME
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value -I../include -Icsrc -Ihost $FLAGS"
# MSD_SRC=path: an alternative smj_msd.hip (e.g. `git show REV:...` of an earlier kernel)
# SRC_DIR=dir: an alternative csrc/ as a whole (e.g. `git archive REV` of an earlier tree)
S=${SRC_DIR:-csrc}
[ "$S" != csrc ] && H="$H -I$S"
for f in smj_kernels smj_api smj_host; do $H -c $S/$f.hip -o build/v_$NAME/$f.o & done
$H -c ${MSD_SRC:-$S/smj_msd.hip} -o build/v_$NAME/smj_msd.o & wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsmj_hip.so build/v_$NAME/*.o -Wl,-soname,libsmj_hip.so
echo built $OUT/libsmj_hip.so
