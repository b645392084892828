#!/usr/bin/env python3
"""Round-6 stress shapes at partitioned-mode sizes: two 2-column tables of
ROWS rows each (above the library's part size, so the one-pass partition and
the per-part pipelines run), checked bit for bit against the CPU port
(oracle/cpu_mt.cpp: the same select -> stable sort -> zip join on 16 host
threads) -- the sorted tables and the joined rows.

    python tools/big_stress.py [rows]      (default 2e8)
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import torch  # noqa: E402

import oracle  # noqa: E402
from smj import ops  # noqa: E402

I64 = np.iinfo(np.int64)


def tables(kind, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for x in range(2):
        if kind == "farout":  # dense keys, 1 % anywhere in int64, the extremes
            k = rng.integers(0, 3 * n, size=n, dtype=np.int64)
            m = rng.random(n) < 0.01
            k[m] = rng.integers(I64.min, I64.max, size=int(m.sum()), dtype=np.int64, endpoint=True)
        else:  # "clust": 1024 clusters 2^40 apart, 2^20 wide, 0.1 % anywhere
            k = (rng.integers(0, 1024, size=n, dtype=np.int64) - 512) * (1 << 40) + rng.integers(0, 1 << 20, size=n)
            m = rng.random(n) < 0.001
            k[m] = rng.integers(I64.min, I64.max, size=int(m.sum()), dtype=np.int64, endpoint=True)
        k[rng.choice(n, 1000, replace=False)] = I64.min
        k[rng.choice(n, 1000, replace=False)] = I64.max
        t = np.empty((n, 2), dtype=np.int64)
        t[:, 0] = k
        t[:, 1] = x * (1 << 40) + np.arange(n, dtype=np.int64)
        out.append(t)
    R, S = out
    pick = rng.random(n) < 0.3
    S[pick, 0] = R[rng.integers(0, n, size=int(pick.sum())), 0]
    return R, S


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
    bad = 0
    for kind, seed in (("farout", 1), ("clust", 2)):
        t0 = time.time()
        R, S = tables(kind, n, seed)
        gR, gS, gJ = ops.sort_merge_join(torch.from_numpy(R).cuda(), torch.from_numpy(S).cuda(), 0, 0, None, None)
        torch.cuda.synchronize()
        t1 = time.time()
        info = (ops.msd_segmented(), ops.msd_groups(), ops.msd_stats()[:2])
        secs, rows, (Rs, Ss, J) = oracle.mt_pipeline(R, S, sel=(0, None, 0, None), outputs=True)
        ok = [np.array_equal(gR.cpu().numpy(), Rs), np.array_equal(gS.cpu().numpy(), Ss),
              np.array_equal(gJ.cpu().numpy(), J)]
        bad += not all(ok)
        print(f"{'ok  ' if all(ok) else 'FAIL'} {kind}: {n} x {n} rows, joined {rows[2]}, R/S/J equal {ok}, "
              f"last part's plan {info}, GPU call {t1 - t0:.1f} s (incl. generation and copy), CPU port {secs:.1f} s",
              flush=True)
        del gR, gS, gJ, Rs, Ss, J, R, S
        torch.cuda.empty_cache()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
