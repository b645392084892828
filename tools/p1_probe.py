"""The one-pass partition (msd_part1_kernel through smj_dev_partition_regions)
on a C4-sized table: 1e9 rows into 7 parts (the partitioned mode's split),
timed alone, against a plain device copy of the table (torch) as the
read + write bandwidth reference.  With SMJ_LIB pointing at a build with
-DSMJ_P1_ABL=1 the look-back is skipped (output invalid: timing only).

    python tools/p1_probe.py [rows]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from smj import ops  # noqa: E402


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, float(np.median(ts)) * 1e3


n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
T = ops.gen_uniform(n, seed=1, key_range=3 * n)
sample = T[:, 0][torch.arange(8192, device=T.device) * (n // 8192)].cpu().numpy()  # integer indices: in bounds
bounds = [int(x) for x in np.quantile(sample, np.arange(1, 7) / 7.0)]
reg, need = ops.region_capacities(sample, n, bounds)
out = torch.empty((need, 2), dtype=torch.int64, device="cuda")
cnt = torch.empty(len(bounds) + 2, dtype=torch.int64, device="cuda")
ms = timed(lambda: ops.partition_regions(T, bounds, reg, cnt, 0, 0, 5000, out=out))
gb = 2 * n * 16 / 1e9
print(f"partition_regions {n} rows, 7 parts: best {ms[0]:.3f} ms, median {ms[1]:.3f} ms ({gb / ms[0]:.2f} TB/s); "
      f"flag {int(cnt[-1])}", flush=True)
dst = torch.empty_like(T)
ms = timed(lambda: dst.copy_(T))
print(f"device copy {n} rows: best {ms[0]:.3f} ms, median {ms[1]:.3f} ms ({gb / ms[0]:.2f} TB/s)", flush=True)
