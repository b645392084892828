#!/usr/bin/env python3
"""Which inputs lose rows: crafted 2- and 3-column tables with far outliers
and the signed extremes (tools/seg_stress.py's failing shapes), each checked
against the oracle under the wide tier's hand-over limit (debug_wide_maxrun).

    python tools/ext_probe.py [seed ...]     (seeds: seg_stress cases too)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

import oracle  # noqa: E402
from seg_stress import case, first_diff  # noqa: E402
from smj import ops  # noqa: E402

I64 = np.iinfo(np.int64)


def crafted(name, n, cols, outl, nmin_s, nmin_r, nmax):
    rng = np.random.default_rng(len(name) + 31 * n + cols)
    out = []
    for x, pay in ((0, 0), (1, 10 ** 9)):
        k = rng.integers(0, 10 ** 6, size=n, dtype=np.int64)
        if outl:
            m = rng.random(n) < outl
            k[m] = rng.integers(I64.min, I64.max, size=int(m.sum()), dtype=np.int64, endpoint=True)
        nm = nmin_s if x else nmin_r
        k[rng.choice(n, nm, replace=False)] = I64.min
        k[rng.choice(n, nmax, replace=False)] = I64.max
        t = rng.integers(-1000, 1000, size=(n, cols), dtype=np.int64)
        t[:, 0] = k
        t[:, 1] = pay + np.arange(n)
        out.append(t)
    return name, cols, 0, out[0], out[1], None


def check(name, cols, kc, R, S, sel):
    gR, gS, gJ = ops.sort_merge_join(torch.from_numpy(R).cuda(), torch.from_numpy(S).cuda(), kc, kc, sel, None)
    torch.cuda.synchronize()
    info = (ops.msd_segmented(), ops.msd_groups(), ops.msd_stats()[:2])
    Rs = oracle.select_sort(R, kc, sel[0] if sel else 0, sel[1] if sel else None)
    Ss = oracle.select_sort(S, kc, 0, None)
    J = oracle.join(Rs, Ss, kc, kc)
    d = [first_diff("R", gR.cpu().numpy(), Rs.reshape(-1, cols), kc),
         first_diff("S", gS.cpu().numpy(), Ss.reshape(-1, cols), kc),
         first_diff("J", gJ.cpu().numpy(), J.reshape(-1, 2 * cols - 1), kc)]
    d = [x for x in d if x]
    print(f"{'FAIL' if d else 'ok  '} {name}: seg/groups/single,big {info}", flush=True)
    for x in d:
        print("      " + x, flush=True)


def main():
    cases = [crafted("uniform", 400_000, 2, 0, 0, 0, 0),
             crafted("min45S", 400_000, 2, 0, 45, 0, 0),
             crafted("outl1%", 400_000, 2, 0.01, 0, 0, 0),
             crafted("outl1%+min45S", 400_000, 2, 0.01, 45, 0, 0),
             crafted("outl1%+min45S+max", 400_000, 2, 0.01, 45, 20, 30),
             crafted("outl1%+min45S cols3", 400_000, 3, 0.01, 45, 0, 0),
             crafted("outl0.1%+min45S", 400_000, 2, 0.001, 45, 0, 0),
             crafted("outl1%+min2S", 400_000, 2, 0.01, 2, 0, 0)]
    for s in sys.argv[1:]:
        layout, cols, kc, R, S, sel = case(int(s))
        cases.append((f"seed{s} {layout}", cols, kc, R, S, sel))
    for wm in (-1, 0, 254):
        print(f"== debug_wide_maxrun({wm})", flush=True)
        ops.debug_wide_maxrun(wm)
        for c in cases:
            check(*c)


if __name__ == "__main__":
    main()
