#!/bin/bash
# msd_final ablation: SMJ_DEBUG_MSD bits (1 = stamps, 2 = no radix passes,
# 4 = no sorted-row output, 8 = no join emit, 16 = no join search); timing only
for b in 1 3 5 9 17 25 29 31; do
  echo "== SMJ_DEBUG_MSD=$b"
  SMJ_DEBUG_MSD=$b timeout -k 10 120 python tools/msd_phases.py 2>&1 | grep -v amdgpu | head -3 || exit 1
done
