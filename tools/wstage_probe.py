import sys, os
sys.path.insert(0, "pim-sort-merge-join_amd")
import torch
from smj import ops
for n, kr in ((50_000_000, 150_000_000), (100_000_000, 300_000_000)):
    R = ops.gen_uniform(n, seed=1, key_range=kr); S = ops.gen_uniform(n, seed=2, key_range=kr)
    ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000)); torch.cuda.synchronize()
    print(n, kr, "groups", ops.msd_groups(), "wstage", ops.msd_wstage(), flush=True)
    del R, S
n = 1_000_000_000
R = ops.gen_uniform(n, seed=1, key_range=3 * n); S = ops.gen_uniform(n, seed=2, key_range=3 * n)
ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000)); torch.cuda.synchronize()
print("c4 last part groups", ops.msd_groups(), "wstage", ops.msd_wstage(), flush=True)
