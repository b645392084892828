"""Multi-GPU step costs on one GPU (C3 tables, 1e8 rows each):
  - the partition step: smj_dev_partition_count + _scatter vs the one-call
    smj_dev_partition, 31 splitters (8 ranks x 4 stages);
  - the fused local pipeline on 1/K of the rows (what one stage of
    smj/dist.py runs), K = 1, 2, 4, 8.
python tools/part_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch  # noqa: E402

from smj import ops  # noqa: E402


def timed(fn, reps=4):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


n = 100_000_000
T = ops.gen_uniform(n, seed=1, key_range=3 * n)
bounds = torch.tensor(sorted(int(x) for x in torch.linspace(1e7, 2.9e8, 31).tolist()), dtype=torch.int64,
                      device=T.device)
out = torch.empty_like(T)
counts, _ = ops.partition_count(T, bounds, 0, 0, 5000)
print(f"partition_count {timed(lambda: ops.partition_count(T, bounds, 0, 0, 5000)):.3f} ms", flush=True)
print(f"partition_scatter {timed(lambda: ops.partition_scatter(T, bounds, counts, 0, 0, 5000, out=out)):.3f} ms",
      flush=True)
print(f"partition (fused) {timed(lambda: ops.partition(T, bounds, 0, 0, 5000, out=out)):.3f} ms", flush=True)
c2, got = ops.partition(T, bounds, 0, 0, 5000, out=out)
ref = ops.partition_scatter(T, bounds, counts, 0, 0, 5000)
assert c2 == counts and torch.equal(got, ref), "fused partition differs"
del ref, out
S = ops.gen_uniform(n, seed=2, key_range=3 * n)
for K in (1, 2, 4, 8):
    m = n // K
    Rk, Sk = T[:m].contiguous(), S[:m].contiguous()
    Rs, Ss = torch.empty_like(Rk), torch.empty_like(Sk)
    J = torch.empty((m, 3), dtype=torch.int64, device=T.device)
    ms = timed(lambda: ops.sort_merge_join(Rk, Sk, 0, 0, None, None, R_sorted=Rs, S_sorted=Ss, out=J))
    print(f"local pipeline K={K}: {m} rows/table {ms:.3f} ms/stage, x{K} = {ms * K:.3f} ms", flush=True)
    del Rk, Sk, Rs, Ss, J
