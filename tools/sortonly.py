"""Run select_sort on the C3 table a few times (for rocprofv3 PMC passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch
from smj import ops
n = int(os.environ.get("ROWS", "100000000"))
R = ops.gen_uniform(n, seed=1, key_range=3 * n)
out = torch.empty_like(R)
for _ in range(int(os.environ.get("REPS", "2"))):
    ops.select_sort(R, 0, 0, 5000, out=out)
torch.cuda.synchronize()
print("ok")
