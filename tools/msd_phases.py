"""Phase breakdown of msd_final (SMJ_DEBUG_MSD=1 stamps) on the C3 workload.

    python tools/msd_phases.py            (ROWS=1e8 by default)
"""
import ctypes
import os
import sys
import time

os.environ["SMJ_DEBUG_MSD"] = os.environ.get("SMJ_DEBUG_MSD", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch  # noqa: E402

from smj import _lib, ops  # noqa: E402

lib = _lib.load()
n = int(float(os.environ.get("ROWS", "1e8")))
if os.environ.get("WORKLOAD") == "c5":  # C5's Zipf(0.9) tables, 1e8 x 1e9 (partitioned mode)
    R = ops.gen_zipf(100_000_000, seed=3, domain=100_000_000, theta=0.9)
    S = ops.gen_zipf(1_000_000_000, seed=4, domain=100_000_000, theta=0.9)
else:
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
bufs = [torch.empty_like(R), torch.empty_like(S), torch.empty((R.shape[0], 3), dtype=torch.int64, device=R.device)]
ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), *bufs)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 24)()
lib.smj_debug_msd_phases(buf)  # reset
reps = 3
t0 = time.perf_counter()
for _ in range(reps):
    ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), *bufs)
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t0) / reps * 1e3:.3f} ms/step (with stamps)")
lib.smj_debug_msd_phases(buf)
groups = buf[9]
names = ["first group", "next group offs", "stage+sort", "next lists+rows", "out+join", "loop barrier",
         "", "", "slow path"]
tot = sum(buf[k] for k in range(9))
print(f"groups {groups}; cycles/group (thread0 view, s_memtime):")
for k in range(9):
    if names[k]:
        print(f"  {names[k]:18s} {buf[k] / max(groups, 1):10.0f}  {100 * buf[k] / max(tot, 1):5.1f}%")
print(f"  total              {tot / max(groups, 1):10.0f}")
sub = ["sort: stage+hist", "sort: scan", "sort: scatter", "sort: dup fix-up", "issue: lists", "issue: row loads"]
for k in range(6):
    print(f"    {sub[k]:18s} {buf[10 + k] / max(groups, 1):10.0f}")
tiles = buf[23]
pb = ["list + lookups", "row loads issued", "rank (loads land)", "digit starts", "stage + offs", "stores issued"]
print(f"part_b tiles {tiles}; cycles/tile (thread0 view):")
tot = sum(buf[16 + k] for k in range(6))
for k in range(6):
    print(f"  {pb[k]:18s} {buf[16 + k] / max(tiles, 1):10.0f}  {100 * buf[16 + k] / max(tot, 1):5.1f}%")
print(f"  total              {tot / max(tiles, 1):10.0f}")
sub = ["stage + count", "bin scan", "place (scatter / LSD)", "equal-key rounds", "next lists", "next gathers"]
stot = sum(buf[10 + k] for k in range(6))
print("staged sort sub-phases (cycles/group):")
for k in range(6):
    print(f"  {sub[k]:22s} {buf[10 + k] / max(groups, 1):10.0f}  {100 * buf[10 + k] / max(stot, 1):5.1f}%")
