"""Group statistics of one C5 part (the last pipeline call of a C5 step):
dense groups, radix / wide / in-LDS-LSD tiers, single-key and oversized
groups, selected rows per table.

    python tools/c5_groups.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch  # noqa: E402

from smj import ops  # noqa: E402

R = ops.gen_zipf(100_000_000, seed=3, domain=100_000_000, theta=0.9)
S = ops.gen_zipf(1_000_000_000, seed=4, domain=100_000_000, theta=0.9)
ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000))
torch.cuda.synchronize()
g = ops.msd_groups()
st = ops.msd_stats()
print(json.dumps({"dense_groups": g[0], "radix_tier": g[1], "wide_tier": g[2], "lds_lsd": g[3] if len(g) > 3 else None,
                  "single_key": st[0], "oversized": st[1], "rows_R": st[2], "rows_S": st[3],
                  "bigdev": ops.msd_bigdev() if hasattr(ops, "msd_bigdev") else None}))
