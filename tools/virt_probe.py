"""Partitioned mode at C3 size: the pipeline's per-stage cost when the tables
are first cut into P key-range parts (force_parts = 1, 2, 4, 8, 16) against
the plain pipeline (0).

Round 3 used it on a level-1 split that part_a read back as virtual tables
(profiles/r03/r03g_virtual_parts_probe.txt: part_a 1.29 ms plain, 1.53 ms
with one part, 2.11 ms with eight -- each virtual tile gathering ~P segments
from P split tiles -- so C4 went from 68 to 71 ms and the split was dropped);
it now measures the contiguous partition (partition_hist / _scatter).

    python tools/virt_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))

import torch  # noqa: E402

from smj import ops  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    bufs = dict(R_sorted=torch.empty_like(R), S_sorted=torch.empty_like(S),
                out=torch.empty((n, 3), dtype=torch.int64, device=R.device))
    res = {}
    for parts in (0, 1, 2, 4, 8, 16):
        ops.force_parts(parts)
        ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), **bufs)
        torch.cuda.synchronize()
        ops.prof_enable(True)
        ops.prof_report()
        for _ in range(3):
            ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), **bufs)
        torch.cuda.synchronize()
        ops.prof_enable(False)
        pr = ops.prof_report()
        res[parts] = {k: round(v["ms"] / 3, 4) for k, v in pr.items() if v["ms"] / 3 > 0.02}
        print(parts, res[parts], flush=True)
    ops.force_parts(0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
