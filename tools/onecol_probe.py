"""How much of the C3 step is row bytes: the same keys as 1-column tables
(8-B rows through every pass) against the 2-column tables (16-B rows).
Prints ms per call and the per-stage scopes of both."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch  # noqa: E402

from smj import ops  # noqa: E402

n = int(float(os.environ.get("ROWS", "1e8")))
R = ops.gen_uniform(n, seed=1, key_range=3 * n)
S = ops.gen_uniform(n, seed=2, key_range=3 * n)
R1, S1 = R[:, :1].contiguous(), S[:, :1].contiguous()
for name, (a, b) in (("2col", (R, S)), ("1col", (R1, S1)), ("2col", (R, S)), ("1col", (R1, S1))):
    bufs = (torch.empty_like(a), torch.empty_like(b), torch.empty((n, 2 * a.shape[1] - 1), dtype=torch.int64,
                                                                   device=a.device))
    for _ in range(2):
        ops.sort_merge_join(a, b, 0, 0, (0, 5000), (0, 5000), *bufs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        ops.sort_merge_join(a, b, 0, 0, (0, 5000), (0, 5000), *bufs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10 * 1e3
    ops.prof_enable(True)
    ops.prof_report()
    for _ in range(3):
        ops.sort_merge_join(a, b, 0, 0, (0, 5000), (0, 5000), *bufs)
    torch.cuda.synchronize()
    ops.prof_enable(False)
    pr = ops.prof_report()
    print(name, f"{dt:.3f} ms", {k: round(v["ms"] / 3, 3) for k, v in pr.items() if v["ms"] / 3 > 0.05}, flush=True)
