#!/usr/bin/env python3
"""Randomised parity stress of the segmented pass-B digit (clustered keys):
seeded tables of random cluster layouts (cluster count, gap, width, outliers,
duplicates, the signed extremes), sizes, column counts, key columns and
WHEREs, each checked bit for bit against the oracle.  Prints one line per
failing seed and a summary.

    python tools/seg_stress.py [first_seed] [seeds] [seconds]
    python tools/seg_stress.py --seeds=11,25   (those seeds, each failure in detail)
    python tools/seg_stress.py --mixed 0 200   (case_mixed: two shapes, WHEREs on both, partitioned mode)
    python tools/seg_stress.py --host 0 200    (the mixed cases through smj_sort_merge_join, host pointers)
    python tools/seg_stress.py --typed 0 200   (the mixed cases with T = uint64 / double)
    python tools/seg_stress.py --hostbig 0 40  (host tables of 3M-9M rows: several staged chunks)
"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))  # (oracle/oracle.py, as tests/conftest.py has it)

import torch  # noqa: E402

import oracle  # noqa: E402
from smj import ops  # noqa: E402

I64 = np.iinfo(np.int64)


def table(rng, n, cols, key_col, pay0, layout):
    nclu, gap_bits, width, outl, dup = layout
    u = rng.integers(0, width, size=n, dtype=np.int64)
    c = rng.integers(0, nclu, size=n, dtype=np.int64)
    k = (c - nclu // 2) * (np.int64(1) << np.int64(gap_bits)) + u
    if dup:
        k = k - (k % dup)
    if outl:
        m = rng.random(n) < outl
        k[m] = rng.integers(I64.min, I64.max, size=int(m.sum()), dtype=np.int64, endpoint=True)
    if rng.random() < 0.2:
        k[rng.random(n) < 0.001] = I64.max
        k[rng.random(n) < 0.001] = I64.min
    t = rng.integers(-1000, 1000, size=(n, cols), dtype=np.int64)
    t[:, key_col] = k
    if cols > 1:
        t[:, (key_col + 1) % cols] = pay0 + np.arange(n)
    return t


def case(seed):
    rng = np.random.default_rng(10_000 + seed)
    nclu = int(rng.choice([2, 3, 8, 64, 300, 1024, 5000]))
    gap_bits = int(rng.integers(20, 58))
    gap_bits = min(gap_bits, 62 - int(np.ceil(np.log2(nclu))))
    width = int(rng.choice([10, 1000, 10 ** 5, 10 ** 6, 1 << 20]))
    layout = (nclu, gap_bits, min(width, 1 << (gap_bits - 1)), float(rng.choice([0, 0, 0.001, 0.01])),
              int(rng.choice([0, 0, 0, 7, 1000])))
    cols = int(rng.choice([1, 2, 2, 2, 3]))
    kc = int(rng.integers(0, cols))
    nr, ns = (int(rng.integers(20_000, 700_000)) for _ in range(2))
    R = table(rng, nr, cols, kc, 0, layout)
    S = table(rng, ns, cols, kc, 10 ** 9, layout)
    pick = rng.random(ns) < 0.3
    S[pick, kc] = R[rng.integers(0, nr, size=int(pick.sum())), kc]
    sel = None
    if rng.random() < 0.3 and cols > 1:
        sc = (kc + 1) % cols
        sel = (sc, int(np.sort(R[:, sc])[int(rng.integers(0, nr))]))
    return layout, cols, kc, R, S, sel


def case_mixed(seed, big=False):
    """Mixed shapes: R and S of their own column counts (1-5) and key
    columns, a WHERE on either, tiny to 2M-row tables, and the partitioned
    mode forced on some seeds (parts)."""
    rng = np.random.default_rng(50_000 + seed)
    nclu = int(rng.choice([1, 2, 8, 64, 1024]))
    gap_bits = min(int(rng.integers(10, 58)), 62 - int(np.ceil(np.log2(max(nclu, 2)))))
    width = int(rng.choice([10, 1000, 10 ** 6, 1 << 30]))
    layout = (nclu, gap_bits, min(width, 1 << (gap_bits - 1)), float(rng.choice([0, 0, 0.001, 0.01])),
              int(rng.choice([0, 0, 7])))
    c1, c2 = (int(rng.choice([1, 2, 2, 3, 5])) for _ in range(2))
    k1, k2 = int(rng.integers(0, c1)), int(rng.integers(0, c2))
    nr, ns = (int(rng.choice([0, 1, 100, 5000, 300_000, 2_000_000])) if rng.random() < 0.3
              else int(rng.integers(20_000, 900_000)) for _ in range(2))
    if big:  # several of the staged host path's 3,440,640-row chunks, ragged last ones
        nr, ns = (int(rng.integers(3_000_000, 9_000_000)) for _ in range(2))
    R = table(rng, nr, c1, k1, 0, layout)
    S = table(rng, ns, c2, k2, 10 ** 9, layout)
    if nr and ns:
        pick = rng.random(ns) < 0.3
        S[pick, k2] = R[rng.integers(0, nr, size=int(pick.sum())), k1]
    sels = []
    for T, c, k in ((R, c1, k1), (S, c2, k2)):
        sel = None
        if rng.random() < 0.3 and c > 1 and len(T):
            sc = (k + 1) % c
            sel = (sc, int(np.sort(T[:, sc])[int(rng.integers(0, len(T)))]))
        sels.append(sel)
    parts = int(rng.choice([0, 0, 0, 2, 3])) if nr + ns > 100_000 else 0
    return (layout, parts), (c1, c2), (k1, k2), R, S, tuple(sels)


def first_diff(name, g, o, kc):
    """One line on how the device table g differs from the oracle's o."""
    if g.shape != o.shape:
        return f"{name}: rows {g.shape[0]} vs oracle {o.shape[0]}"
    bad = np.nonzero((g != o).any(axis=1))[0]
    if not len(bad):
        return None
    i = int(bad[0])
    srt = bool((np.diff(g[:, kc]) >= 0).all()) if name != "J" else None
    same = np.array_equal(g[np.lexsort(g.T[::-1])], o[np.lexsort(o.T[::-1])])
    return (f"{name}: {len(bad)} rows differ, first {i}: {g[i].tolist()} vs {o[i].tolist()}"
            f" (prev {o[max(i - 1, 0)].tolist()}) sorted {srt} same-multiset {same}")


class Block(ctypes.Structure):  # user.h's block_t (smj.h)
    _fields_ = [("table_num", ctypes.c_int), ("col_num", ctypes.c_int), ("row_num", ctypes.c_int)]


class Timing(ctypes.Structure):
    _fields_ = [("cpu_gpu_ms", ctypes.c_double), ("gpu_ms", ctypes.c_double), ("gpu_cpu_ms", ctypes.c_double)]


def host_join(lib, R, S, k1, k2, s1, s2):
    """smj_sort_merge_join on host tables, as app.c calls it (a WHERE on both
    tables always: None -> row[0] > INT64_MIN)."""
    c1, c2 = R.shape[1], S.shape[1]
    R, S = np.ascontiguousarray(R), np.ascontiguousarray(S)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    res, rows, tm = ctypes.c_void_p(), ctypes.c_int64(0), Timing()
    rc = lib.smj_sort_merge_join(ctypes.byref(Block(0, c1, len(R))), p(R), ctypes.byref(Block(1, c2, len(S))), p(S),
                                 s1[0], s1[1], s2[0], s2[1], k1, k2, ctypes.byref(res), ctypes.byref(rows),
                                 ctypes.byref(tm))
    if rc != 0:
        raise RuntimeError(f"smj_sort_merge_join -> {rc}")
    tc = c1 + c2 - 1
    got = np.empty((0, tc), dtype=np.int64)
    if res.value:
        got = np.ctypeslib.as_array(ctypes.cast(res, ctypes.POINTER(ctypes.c_int64)),
                                    shape=(rows.value * tc,)).copy().reshape(-1, tc)
        libc = ctypes.CDLL(None)
        libc.free.argtypes = [ctypes.c_void_p]
        libc.free(res)
    return got


_LIB = None


def check_seed(seed, mode="plain"):
    """One seed of a mode (plain / mixed / host / typed): (diffs, description,
    segmented buckets, plan info).  diffs is empty when the device output
    equals the oracle's bit for bit."""
    global _LIB
    typed, hostp = mode == "typed", mode in ("host", "hostbig")
    if mode == "plain":
        layout, cols, kc, R, S, sel = case(seed)
        parts, c1, c2, k1, k2, sel2 = 0, cols, cols, kc, kc, None
    else:
        (layout, parts), (c1, c2), (k1, k2), R, S, (sel, sel2) = case_mixed(seed, mode == "hostbig")
    nr, ns = len(R), len(S)
    if hostp:  # app.c always selects: None -> row[0] > INT64_MIN
        sel = sel or (0, int(I64.min))
        sel2 = sel2 or (0, int(I64.min))
        parts = 0
        if _LIB is None:
            from smj import _lib
            _LIB = _lib.load()
            assert _LIB.smj_init(1) >= 1
    kt = (1 + seed % 2) if typed else 0  # T = uint64 (odd seeds) / double (even seeds)
    if kt == 1:  # the int64 patterns as uint64 (negative keys wrap past 2^63); WHERE values likewise
        sel = sel and (sel[0], sel[1] % (1 << 64))
        sel2 = sel2 and (sel2[0], sel2[1] % (1 << 64))
    elif kt == 2:  # the same values as doubles (clusters up to 2^62 round to 53 bits: duplicates)
        R, S = R.astype(np.float64), S.astype(np.float64)
        sel = sel and (sel[0], float(sel[1]))
        sel2 = sel2 and (sel2[0], float(sel2[1]))
    desc = (f"layout {layout} cols {c1}/{c2} keys {k1}/{k2} n {nr}/{ns} sel {sel}/{sel2} parts {parts}"
            + (f" T {kt}" if kt else ""))
    cuda = (lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda())
    gR = gS = gJ = None
    ops.force_parts(parts)
    try:
        if hostp:
            try:
                gJ = torch.from_numpy(host_join(_LIB, R.reshape(-1, c1), S.reshape(-1, c2), k1, k2, sel, sel2))
            except RuntimeError as e:  # an error code: a failure of this seed, not of the run
                desc += f" ({e})"
        else:
            gR, gS, gJ = ops.sort_merge_join(cuda(R), cuda(S), k1, k2, sel, sel2, key_type=kt)
        torch.cuda.synchronize()
    finally:
        ops.force_parts(0)
    nseg = ops.msd_segmented()
    info = (ops.msd_packb(), ops.msd_groups(), ops.msd_stats())
    if kt:
        bits = (lambda a: np.ascontiguousarray(a).view(np.int64))
        Rs = bits(oracle.select_sort_t(R.reshape(-1, c1), kt, k1, *(sel or (0, None))))
        Ss = bits(oracle.select_sort_t(S.reshape(-1, c2), kt, k2, *(sel2 or (0, None))))
        J = bits(oracle.join_t(Rs.reshape(-1, c1), Ss.reshape(-1, c2), kt, k1, k2))
        gR, gS, gJ = (t.view(torch.int64) for t in (gR, gS, gJ))
    else:
        Rs = oracle.select_sort(R.reshape(-1, c1), k1, sel[0] if sel else 0, sel[1] if sel else None)
        Ss = oracle.select_sort(S.reshape(-1, c2), k2, sel2[0] if sel2 else 0, sel2[1] if sel2 else None)
        J = oracle.join(Rs.reshape(-1, c1), Ss.reshape(-1, c2), k1, k2)
    diffs = [first_diff("J", gJ.cpu().numpy(), J.reshape(-1, c1 + c2 - 1), k1) if gJ is not None else "error code"]
    if not hostp:
        diffs += [first_diff("R", gR.cpu().numpy(), Rs.reshape(-1, c1), k1),
                  first_diff("S", gS.cpu().numpy(), Ss.reshape(-1, c2), k2)]
    return [d for d in diffs if d], desc, nseg, info


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    seeds = None
    for a in sys.argv[1:]:
        if a.startswith("--seeds="):
            seeds = [int(x) for x in a[8:].split(",")]
    first = int(args[0]) if len(args) > 0 else 0
    count = int(args[1]) if len(args) > 1 else 100
    budget = float(args[2]) if len(args) > 2 else 240.0
    mode = next((m for m in ("mixed", "hostbig", "host", "typed") if f"--{m}" in sys.argv), "plain")
    t0 = time.time()
    bad = done = seg_runs = 0
    for seed in seeds if seeds is not None else range(first, first + count):
        if time.time() - t0 > budget:
            break
        diffs, desc, nseg, info = check_seed(seed, mode)
        seg_runs += nseg > 0
        done += 1
        if done % 10 == 0:
            print(f"  {done} seeds, {bad} failures, {time.time() - t0:.0f} s", flush=True)
        if diffs:
            bad += 1
            print(f"FAIL seed {seed}: {desc} segmented {nseg}", flush=True)
            if seeds is not None:
                print(f"    packb {info[0]} groups {info[1]} stats {info[2]}", flush=True)
                for d in diffs:
                    print("    " + d, flush=True)
    print(f"seg_stress: {done} seeds ({mode}), {bad} failures, {seg_runs} with segmented buckets, "
          f"{time.time() - t0:.0f} s", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
