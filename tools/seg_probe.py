#!/usr/bin/env python3
"""Clustered-key probe of the segmented pass-B digit (MsdSeg): 1e8 x 1e8
tables with keys in dense clusters far apart, timed with the digit on and off
(SMJ_SEG=0); prints ms per call (median of 5 after 2 warm-ups), the tier
counts and the per-kernel times of one profiled call.  Correctness: the GPU
tests (tests/test_gpu_msd.py -k clustered)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))

import torch  # noqa: E402

from smj import ops  # noqa: E402


def tables(n, kind):
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    for t in (R, S):
        u = t[:, 0]
        if kind == "clust64":
            t[:, 0] = (u % 64) * (1 << 40) + u // 64
        elif kind == "clust1k":
            t[:, 0] = (u % 1024) * (1 << 33) + u // 1024
        elif kind == "clust3":
            r = (u * 2654435761) % 100
            t[:, 0] = torch.where(r < 90, 0, torch.where(r < 99, 1 << 50, 1 << 51)) + u
    return R, S


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    kinds = sys.argv[2:] or ["clust64", "clust1k", "clust3"]
    for kind in kinds:
        R, S = tables(n, kind)
        bR, bS = torch.empty_like(R), torch.empty_like(S)
        J = torch.empty((n, 3), dtype=torch.int64, device=R.device)
        for seg in ("1", "0"):
            os.environ["SMJ_SEG"] = seg
            times = []
            for i in range(7):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                _, _, j = ops.sort_merge_join(R, S, 0, 0, None, None, R_sorted=bR, S_sorted=bS, out=J)
                torch.cuda.synchronize()
                times.append((time.perf_counter() - t0) * 1e3)
            times = sorted(times[2:])
            line = (f"{kind:8s} seg={seg} {times[len(times) // 2]:8.3f} ms  joined {j.shape[0]:>11,d}  "
                    f"segmented {ops.msd_segmented()}  groups/radix/wide/lsd {ops.msd_groups()}  "
                    f"wstage {ops.msd_wstage()}  single/big {ops.msd_stats()[:2]}  bigdev {ops.msd_bigdev()}")
            if seg == "1":  # the oversized groups left (size histogram, first few: stderr)
                os.environ["SMJ_DEBUG_BIG"] = "1"
                ops.sort_merge_join(R, S, 0, 0, None, None, R_sorted=bR, S_sorted=bS, out=J)
                torch.cuda.synchronize()
                os.environ.pop("SMJ_DEBUG_BIG")
            ops.prof_enable(True)
            ops.sort_merge_join(R, S, 0, 0, None, None, R_sorted=bR, S_sorted=bS, out=J)
            rep = ops.prof_report()
            ops.prof_enable(False)
            ks = {k: round(v["ms"], 3) for k, v in (json.loads(rep) if isinstance(rep, str) else rep).items()
                  if v["ms"] > 0.05}
            print(line, flush=True)
            print("   ", ks, flush=True)
        del R, S, bR, bS, J
        torch.cuda.empty_cache()
    os.environ.pop("SMJ_SEG", None)


if __name__ == "__main__":
    main()
