import sys
sys.path.insert(0, "pim-sort-merge-join_amd")
import torch
from smj import ops, _lib
def rep(tag):
    free, tot = torch.cuda.mem_get_info()
    print(f"{tag:40s} lib {ops.scratch_bytes()/2**30:7.1f} GiB  torch {torch.cuda.memory_allocated()/2**30:6.1f}  free {free/2**30:6.1f}", flush=True)
SEL = 5000
for n in (100_000_000,):
    R = ops.gen_wide(n, seed=1); S = ops.gen_wide(n, seed=2, plant_seed=1, plant_rows=n)
    g = ops.sort_merge_join(R, S, 0, 0, (0, -(1 << 63)), (0, -(1 << 63))); torch.cuda.synchronize(); rep("c3w"); del R, S, g
n = 1_000_000_000
R = ops.gen_uniform(n, seed=1, key_range=3 * n); S = ops.gen_uniform(n, seed=2, key_range=3 * n)
g = ops.sort_merge_join(R, S, 0, 0, (0, SEL), (0, SEL)); torch.cuda.synchronize(); rep("c4")
ops.trim(); rep("c4 trimmed"); del R, S, g; torch.cuda.empty_cache()
for n, prof in ((292_000_000, False), (559_000_000, False), (292_000_000, True), (559_000_000, True)):
    R = ops.gen_uniform(n, seed=1, key_range=3 * n); S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    ops.prof_enable(prof)
    g = ops.sort_merge_join(R, S, 0, 0, (0, SEL), (0, SEL)); torch.cuda.synchronize()
    ops.prof_enable(False); ops.prof_report()
    rep(f"n={n} prof={prof}"); del R, S, g; torch.cuda.empty_cache()
