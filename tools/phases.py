"""Phase breakdown of the radix scatter kernel (SMJ_DEBUG_PASS=8 stamps)."""
import ctypes, os, sys
os.environ["SMJ_DEBUG_PASS"] = os.environ.get("SMJ_DEBUG_PASS", "8")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch
from smj import ops, _lib
lib = _lib.load()
n = int(os.environ.get("ROWS", "100000000"))
R = ops.gen_uniform(n, seed=1, key_range=3 * n)
out = torch.empty_like(R)
ops.select_sort(R, 0, 0, 5000, out=out); torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 16)()
lib.smj_debug_phase_cycles(buf)  # reset
for _ in range(2):
    ops.select_sort(R, 0, 0, 5000, out=out)
torch.cuda.synchronize()
lib.smj_debug_phase_cycles(buf)
tiles = buf[7]
names = ["zero+B1", "digits+rank", "totals", "scan", "pos+prefetch", "stage+adj", "scatter"]
tot = sum(buf[k] for k in range(7))
print(f"tiles {tiles}; cycles/tile (thread0 view, s_memtime ticks):")
for k in range(7):
    print(f"  {names[k]:14s} {buf[k] / tiles:10.0f}  {100 * buf[k] / tot:5.1f}%")
print(f"  total          {tot / tiles:10.0f}")
