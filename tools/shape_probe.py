#!/usr/bin/env python3
"""Timing probe of the fused pipeline on 1e8 x 1e8 tables of other key shapes
(perf cliffs outside the BASELINE workloads): sorted / reversed / nearly
sorted input, few distinct keys, all-equal keys, clustered keys, keys in
column 1.  Prints ms per call (median of 5 after 2 warm-ups), the tier
counts, and the join row count.  No correctness checks here (the GPU tests
cover the shapes at smaller sizes)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))

import torch  # noqa: E402

from smj import ops  # noqa: E402


def shapes(n):
    dev = "cuda"
    idx = torch.arange(n, device=dev, dtype=torch.int64)
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    yield "uniform [1,3n]", R, S
    Rs = R.clone(); Rs[:, 0] = torch.sort(R[:, 0]).values
    Ss = S.clone(); Ss[:, 0] = torch.sort(S[:, 0]).values
    yield "sorted keys", Rs, Ss
    Rr = Rs.clone(); Rr[:, 0] = Rs[:, 0].flip(0)
    Sr = Ss.clone(); Sr[:, 0] = Ss[:, 0].flip(0)
    yield "reversed keys", Rr, Sr
    del Rs, Ss, Rr, Sr
    for d in (1000, 100_000):
        Rd = R.clone(); Rd[:, 0] = R[:, 0] % d
        Sd = S.clone(); Sd[:, 0] = S[:, 0] % d
        yield f"{d} distinct keys", Rd, Sd
        del Rd, Sd
    Re = R.clone(); Re[:, 0] = 7
    Se = S.clone(); Se[:, 0] = 7
    yield "all keys equal", Re, Se
    del Re, Se
    # clustered: 64 dense runs of keys far apart (gaps of 2^40)
    Rc = R.clone(); Rc[:, 0] = (R[:, 0] % 64) * (1 << 40) + (R[:, 0] // 64)
    Sc = S.clone(); Sc[:, 0] = (S[:, 0] % 64) * (1 << 40) + (S[:, 0] // 64)
    yield "64 key clusters 2^40 apart", Rc, Sc
    del Rc, Sc
    Rk = R.flip(1).contiguous(); Sk = S.flip(1).contiguous()
    yield "key in column 1", Rk, Sk


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    for name, R, S in shapes(n):
        kc = 1 if "column 1" in name else 0
        bR, bS = torch.empty_like(R), torch.empty_like(S)
        J = torch.empty((n, 3), dtype=torch.int64, device=R.device)
        times = []
        for i in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, _, j = ops.sort_merge_join(R, S, kc, kc, None, None, R_sorted=bR, S_sorted=bS, out=J)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        times = sorted(times[2:])
        if os.environ.get("SHAPE_PROF"):  # per-scope times of one more call
            ops.prof_enable(True)
            ops.sort_merge_join(R, S, kc, kc, None, None, R_sorted=bR, S_sorted=bS, out=J)
            rep = ops.prof_report()
            ops.prof_enable(False)
            print("   ", {k: round(v["ms"], 3) for k, v in rep.items() if v["ms"] > 0.05}, flush=True)
        print(f"{name:28s} {times[len(times) // 2]:8.3f} ms  joined {j.shape[0]:>11,d}  groups/radix/wide/lsd "
              f"{ops.msd_groups()}  wstage {ops.msd_wstage()}  single/big {ops.msd_stats()[:2]}  "
              f"packB {ops.msd_packb()}", flush=True)
        del R, S, bR, bS, J
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
