"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit for
bit, on seeded inputs; the reference's golden CSVs end to end through the C
host smj_app; size-independent properties at BASELINE sizes."""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import PKG, case_config, fixture_path

import oracle

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).cuda()


def host(t):
    return t.cpu().numpy()


def rand_table(rng, n, cols, kind, key_col=0):
    if kind == "dups":
        t = rng.integers(-50, 50, size=(n, cols), dtype=np.int64)
    elif kind == "wide":
        t = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=(n, cols), dtype=np.int64,
                         endpoint=True)
    elif kind == "same":
        t = np.full((n, cols), 7, dtype=np.int64)
    elif kind == "uniform":
        t = rng.integers(1, 3 * max(n, 1), size=(n, cols), dtype=np.int64, endpoint=True)
    elif kind == "extremes":
        vals = np.array([np.iinfo(np.int64).min, -1, 0, 1, np.iinfo(np.int64).max], dtype=np.int64)
        t = vals[rng.integers(0, 5, size=(n, cols))]
    else:
        raise ValueError(kind)
    if cols > 1:
        t[:, (key_col + 1) % cols] = np.arange(n)  # payload = row id: makes stability visible
    return t


SORT_CASES = [
    # n, cols, kind, key_col, select (col, val) or None
    (0, 2, "uniform", 0, None), (1, 2, "uniform", 0, None), (63, 2, "dups", 0, None),
    (4095, 2, "uniform", 0, (0, 100)), (4096, 2, "dups", 0, None), (4097, 2, "wide", 0, None),
    (100_000, 2, "uniform", 0, (0, 5000)), (250_001, 2, "dups", 1, (0, 0)), (100_000, 2, "same", 0, None),
    (70_000, 2, "extremes", 0, None), (50_000, 1, "wide", 0, None), (60_000, 3, "uniform", 2, (1, 1000)),
    (90_000, 4, "dups", 3, (2, -10)), (33_333, 5, "wide", 4, None), (40_000, 6, "uniform", 1, (5, 5000)),
    (20_000, 7, "dups", 6, None), (30_000, 8, "uniform", 5, (0, 90000)), (1_000_000, 2, "uniform", 0, (0, 5000)),
    # wider than 8 columns: the index-sort path
    (50_000, 9, "dups", 8, (3, 0)), (70_000, 12, "uniform", 4, None), (20_000, 33, "extremes", 31, (0, 0)),
    (0, 16, "uniform", 0, None),
    # full-range keys through the wide-span staged kernel (one table), a WHERE on the other column
    (500_000, 2, "wide", 0, None), (300_000, 2, "wide", 1, (0, 100_000)),
]


@pytest.mark.parametrize("n,cols,kind,key,sel", SORT_CASES)
def test_select_sort_matches_oracle(gpu, oracle_built, n, cols, kind, key, sel):
    from smj import ops
    rng = np.random.default_rng(n * 31 + cols)
    t = rand_table(rng, n, cols, kind, key)
    got = ops.select_sort(dev(t).reshape(n, cols), key_col=key, select_col=sel[0] if sel else 0,
                          select_val=sel[1] if sel else None)
    ref = oracle.select_sort(t, key, sel[0] if sel else 0, sel[1] if sel else None)
    np.testing.assert_array_equal(host(got), ref.reshape(-1, cols))


@pytest.mark.parametrize("n,cols,sel", [(0, 2, (0, 0)), (5000, 2, (0, 10)), (300_001, 3, (1, 0)),
                                        (100_000, 4, (3, -10 ** 17)), (80_000, 10, (9, 3)), (7_000, 25, (2, -40))])
def test_select_matches_oracle(gpu, oracle_built, n, cols, sel):
    from smj import ops
    rng = np.random.default_rng(5)
    t = rng.integers(-50, 50, size=(n, cols), dtype=np.int64)
    if n:
        t[:, 0] = np.arange(n)
    got = ops.select(dev(t).reshape(n, cols), sel[0], sel[1])
    np.testing.assert_array_equal(host(got), oracle.select(t, sel[0], sel[1]).reshape(-1, cols))


@pytest.mark.parametrize("na,nb,cols,kmax", [(0, 10, 2, 5), (10, 0, 2, 5), (1, 1, 2, 1), (5000, 7000, 2, 20),
                                             (100_000, 33_333, 3, 1000), (4096, 4096, 1, 1 << 50),
                                             (250_000, 250_000, 2, 7), (30_000, 50_000, 11, 100),
                                             (0, 5_000, 9, 3)])
def test_merge_matches_oracle(gpu, oracle_built, na, nb, cols, kmax):
    from smj import ops
    rng = np.random.default_rng(na + nb)
    a = oracle.sort(rng.integers(-kmax, kmax, size=(na, cols), dtype=np.int64), 0)
    b = oracle.sort(rng.integers(-kmax, kmax, size=(nb, cols), dtype=np.int64), 0)
    if cols > 1:
        a[:, 1] = np.arange(na)
        b[:, 1] = 10 ** 9 + np.arange(nb)
    got = ops.merge(dev(a).reshape(na, cols), dev(b).reshape(nb, cols), 0)
    np.testing.assert_array_equal(host(got), oracle.merge(a.reshape(na, cols), b.reshape(nb, cols), 0))


JOIN_CASES = [
    # nr, ns, c1, c2, key1, key2, key domain
    (0, 100, 2, 2, 0, 0, 10), (100, 0, 2, 2, 0, 0, 10), (1, 1, 2, 2, 0, 0, 1), (5000, 5000, 2, 2, 0, 0, 20),
    (100_000, 100_000, 2, 2, 0, 0, 300_000), (70_000, 9_000, 3, 2, 1, 0, 50), (9_000, 70_000, 2, 4, 0, 3, 50),
    (200_000, 150_000, 4, 5, 2, 4, 3), (40_000, 40_000, 1, 1, 0, 0, 1 << 60), (50_000, 60_000, 8, 8, 7, 0, 1000),
    (300_000, 300_000, 2, 2, 0, 0, 1),
    # wider than 8 columns: joined through (key, row id) pairs
    (60_000, 40_000, 9, 2, 3, 0, 500), (20_000, 30_000, 3, 14, 0, 13, 40), (10_000, 10_000, 20, 20, 19, 0, 5),
]


@pytest.mark.parametrize("nr,ns,c1,c2,k1,k2,dom", JOIN_CASES)
def test_join_matches_oracle(gpu, oracle_built, nr, ns, c1, c2, k1, k2, dom):
    from smj import ops
    rng = np.random.default_rng(nr * 7 + ns)
    R = rng.integers(-dom, dom, size=(nr, c1), dtype=np.int64)
    S = rng.integers(-dom, dom, size=(ns, c2), dtype=np.int64)
    if c1 > 1:
        R[:, (k1 + 1) % c1] = np.arange(nr)
    if c2 > 1:
        S[:, (k2 + 1) % c2] = 10 ** 9 + np.arange(ns)
    R = oracle.sort(R, k1)
    S = oracle.sort(S, k2)
    got = ops.join(dev(R).reshape(nr, c1), dev(S).reshape(ns, c2), k1, k2)
    np.testing.assert_array_equal(host(got), oracle.join(R, S, k1, k2).reshape(-1, c1 + c2 - 1))


def test_partition_matches_numpy(gpu):
    from smj import ops
    rng = np.random.default_rng(3)
    t = rng.integers(-1000, 1000, size=(200_001, 3), dtype=np.int64)
    t[:, 1] = np.arange(len(t))
    spl = np.array([-500, -500, 0, 10, 999], dtype=np.int64)
    counts, (mn, mx) = ops.partition_count(dev(t), dev(spl), key_col=0, select_col=2, select_val=-900)
    keep = t[t[:, 2] > -900]
    bucket = np.searchsorted(spl, keep[:, 0], side="left")
    assert counts == np.bincount(bucket, minlength=len(spl) + 1).tolist()
    assert (mn, mx) == (keep[:, 0].min(), keep[:, 0].max())
    got = ops.partition_scatter(dev(t), dev(spl), counts, key_col=0, select_col=2, select_val=-900)
    np.testing.assert_array_equal(host(got), keep[np.argsort(bucket, kind="stable")])


@pytest.mark.parametrize("n,cols,nspl,sv", [(200_001, 3, 63, -900), (1_000_000, 2, 31, None), (1, 2, 5, None),
                                             (50_000, 5, 63, 2000), (3_000_000, 2, 0, -5000)])
def test_partition_fused_matches_numpy(gpu, n, cols, nspl, sv):
    """smj_dev_partition (what smj/dist.py runs): counts + stable scatter in one
    call, up to 63 splitters (64 buckets), duplicate splitters, empty
    selection (sv = 2000 keeps nothing)."""
    from smj import ops
    rng = np.random.default_rng(n + nspl)
    t = rng.integers(-1000, 1000, size=(n, cols), dtype=np.int64)
    t[:, 1] = np.arange(n)
    spl = np.sort(rng.integers(-1100, 1100, size=nspl)).astype(np.int64)
    if nspl > 3:
        spl[2] = spl[1]
    sc = cols - 1
    counts, got = ops.partition(dev(t), dev(spl), key_col=0, select_col=sc, select_val=sv)
    keep = t if sv is None else t[t[:, sc] > sv]
    bucket = np.searchsorted(spl, keep[:, 0], side="left")
    assert counts == np.bincount(bucket, minlength=nspl + 1).tolist()
    np.testing.assert_array_equal(host(got), keep[np.argsort(bucket, kind="stable")])


@pytest.mark.parametrize("n,cols,sv", [(300_001, 2, -900), (0, 2, None), (70_000, 3, 2000), (1, 2, None)])
def test_partition_plan_apply_matches_numpy(gpu, n, cols, sv):
    """smj_dev_partition_plan / _apply (smj/dist.py's two-call partition): the
    counts land in a device tensor without a host sync, the plan survives an
    intervening library call (a fused pipeline call reuses the scratch), and
    apply writes the stable bucket order; in == out is refused."""
    from smj import _lib, ops
    rng = np.random.default_rng(n + 17)
    t = rng.integers(-1000, 1000, size=(n, cols), dtype=np.int64)
    t[:, 1] = np.arange(n)
    bounds = [-600, -1, 0, 0, 17, 400]
    dt = dev(t).reshape(n, cols)
    cnt = torch.zeros(len(bounds) + 1, dtype=torch.int64, device="cuda")
    sc = cols - 1
    plan = ops.partition_plan(dt, bounds, cnt, 0, sc, sv)
    # an intervening pipeline call on other tables
    other = dev(rand_table(np.random.default_rng(1), 50_000, 2, "uniform"))
    ops.sort_merge_join(other, other.clone(), 0, 0, (0, 10), None)
    got = ops.partition_apply(dt, bounds, plan, 0, sc, sv)
    keep = t if sv is None else t[t[:, sc] > sv]
    bucket = np.searchsorted(np.array(bounds), keep[:, 0], side="left")
    assert host(cnt).tolist() == np.bincount(bucket, minlength=len(bounds) + 1).tolist()
    np.testing.assert_array_equal(host(got)[:len(keep)], keep[np.argsort(bucket, kind="stable")])
    if n:
        with pytest.raises(_lib.SmjError):
            ops.partition_apply(dt, bounds, plan, 0, sc, sv, out=dt)


@pytest.mark.parametrize("n,cols,sv,scale", [(300_001, 2, -900, 1.0), (0, 2, None, 1.0), (70_000, 3, 2000, 1.0),
                                             (1, 2, None, 1.0), (250_000, 4, None, 0.4), (1_000_000, 2, None, 1.0)])
def test_partition_regions_matches_numpy(gpu, n, cols, sv, scale):
    """smj_dev_partition_regions (smj/dist.py's one-read partition): bucket b's
    selected rows, stable, at their region start; exact counts; the overflow
    flag when regions are sized below the counts (scale < 1: the rows past a
    region's capacity: that region's contents are unspecified, the other
    regions and all counts stay exact); in == out refused."""
    from smj import _lib, ops
    rng = np.random.default_rng(n + 29)
    t = rng.integers(-1000, 1000, size=(n, cols), dtype=np.int64)
    if n:
        t[:, 1] = np.arange(n)
    bounds = [-600, -1, 0, 0, 17, 400]
    nb = len(bounds) + 1
    dt = dev(t).reshape(n, cols)
    sample = t[:, 0][np.linspace(0, max(n - 1, 0), min(n, 4096)).astype(int)].tolist() if n else []
    reg, need = ops.region_capacities(sample, n, bounds)
    if scale < 1.0:
        caps = [int(c * scale) for c in reg[nb:]]
        reg = [sum(caps[:b]) for b in range(nb)] + caps
    cnt = torch.full((nb + 1,), -1, dtype=torch.int64, device="cuda")
    sc = cols - 1
    out = ops.partition_regions(dt, bounds, reg, cnt, 0, sc, sv)
    keep = t if sv is None else t[t[:, sc] > sv]
    bucket = np.searchsorted(np.array(bounds), keep[:, 0], side="left")
    c = host(cnt)
    assert c[:nb].tolist() == np.bincount(bucket, minlength=nb).tolist()
    over = any(c[b] > reg[nb + b] for b in range(nb))
    assert (c[nb] & 1) == int(over) and (c[nb] & 2) == 0 and over == (scale < 1.0 and n > 0)
    got = host(out)
    for b in range(nb):
        rows = keep[bucket == b]
        if len(rows) <= reg[nb + b]:  # an overflowed region's contents are unspecified (the caller re-partitions)
            np.testing.assert_array_equal(got[reg[b]: reg[b] + len(rows)], rows)
    if n:
        with pytest.raises((_lib.SmjError, ValueError)):  # the C layer (in == out) or the size check first
            ops.partition_regions(dt, bounds, reg, cnt, 0, sc, sv, out=dt)


def test_gen_uniform_matches_oracle(gpu, oracle_built):
    from smj import ops
    got = ops.gen_uniform(1_000_003, row0=12345, seed=2, key_range=3_000_000)
    np.testing.assert_array_equal(host(got), oracle.gen_uniform(1_000_003, 12345, 2, 3_000_000))


def test_gen_wide_matches_oracle(gpu, oracle_built):
    """C3-wide generator: device == oracle restatement, full-range
    keys, and a third of S's rows planted with R's keys."""
    from smj import ops
    n = 1_000_003
    R = host(ops.gen_wide(n, row0=7, seed=1))
    S = host(ops.gen_wide(n, row0=7, seed=2, plant_seed=1, plant_rows=n + 7))
    np.testing.assert_array_equal(R, oracle.gen_wide(n, 7, 1))
    np.testing.assert_array_equal(S, oracle.gen_wide(n, 7, 2, 1, n + 7))
    assert R[:, 0].min() < -(1 << 62) and R[:, 0].max() > (1 << 62)
    Rall = oracle.gen_wide(n + 7, 0, 1)
    frac = np.isin(S[:, 0], Rall[:, 0]).mean()
    assert 0.32 < frac < 0.345, frac


def test_gen_zipf_shape(gpu):
    from smj import ops
    z = host(ops.gen_zipf(2_000_000, seed=3, domain=100_000_000, theta=0.9))
    assert z[:, 0].min() >= 1 and z[:, 0].max() <= 100_000_000
    top = np.bincount(np.unique(z[:, 0], return_inverse=True)[1]).max() / len(z)
    assert 0.012 < top < 0.03  # top key ~1.9 % of rows


def test_gen_zipf_sharded_matches_oracle(gpu, oracle_built):
    """The C5 tables under --gpus W (strong scaling): rank r generates rows
    [r n / W, (r + 1) n / W) with row0 = r n / W.  The shards concatenate to the
    one-GPU table bit for bit, and the device generator equals its C
    restatement (keys differ only if pow() rounded differently: counted, at
    most 1 in 1e5 rows)."""
    from smj import ops
    n, W = 2_000_003, 8
    full = host(ops.gen_zipf(n, seed=4, domain=100_000_000, theta=0.9))
    parts = np.concatenate([host(ops.gen_zipf(n * (r + 1) // W - n * r // W, row0=n * r // W, seed=4,
                                              domain=100_000_000, theta=0.9)) for r in range(W)])
    np.testing.assert_array_equal(full, parts)
    from smj import _lib
    ref = oracle.gen_zipf(n, 0, seed=4, domain=100_000_000, theta=0.9,
                          zeta=_lib.load().smj_zipf_zeta(100_000_000, 0.9))
    np.testing.assert_array_equal(full[:, 1], ref[:, 1])
    assert int((full[:, 0] != ref[:, 0]).sum()) <= n // 100_000


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


@pytest.mark.parametrize("case", ["bundled_100k", "test_10k", "test_10k_key1_sel2", "test_10k_key3_key2", "kat_all",
                                  "kat_sel100", "kat_default", "dup_heavy", "dup_heavy_sel", "empty_select",
                                  "all_same_key", "empty_table", "single_rows", "atoi_edge", "wide_mixed",
                                  "neg_wide", "wide12", "wide20_9", "wide9_20"])
def test_smj_app_result_csv_bit_exact(gpu, manifest, golden_dir, tmp_path, case):
    """The C host (drop-in for app.c) on the reference's CSVs: result.csv
    byte-identical to the reference cpu_app.c output."""
    e = manifest["cases"][case]
    sel, keys = case_config(e, manifest["user_h_defaults"])
    out = str(tmp_path / "result.csv")
    cmd = [os.path.join(PKG, "bin", "smj_app"), fixture_path(golden_dir, e["inputs"][0]),
           fixture_path(golden_dir, e["inputs"][1]), "-o", out, "--select", *map(str, sel), "--keys", *map(str, keys)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=120)
    assert sha(out) == e["sha256"], case


def test_host_pointer_api(gpu, oracle_built):
    """smj_select / smj_sort / smj_merge / smj_join / smj_sort_merge_join via ctypes
    (the calls a reference-side FFI stub would make)."""
    from smj import _lib
    lib = _lib.load()
    assert lib.smj_init(1) >= 1

    class Block(ctypes.Structure):
        _fields_ = [("table_num", ctypes.c_int), ("col_num", ctypes.c_int), ("row_num", ctypes.c_int)]

    rng = np.random.default_rng(9)
    R = rng.integers(0, 3000, size=(10_000, 3), dtype=np.int64)
    S = rng.integers(0, 3000, size=(8_000, 2), dtype=np.int64)
    R[:, 1] = np.arange(len(R))
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    bR, bS = Block(0, 3, len(R)), Block(1, 2, len(S))

    out = np.empty_like(R)
    m = ctypes.c_int(0)
    _lib.check(lib.smj_select(ctypes.byref(bR), p(R), p(out), 0, 1500, ctypes.byref(m)), "smj_select")
    np.testing.assert_array_equal(out[: m.value], oracle.select(R, 0, 1500))

    Rs = R.copy()
    _lib.check(lib.smj_sort(ctypes.byref(bR), p(Rs), 0), "smj_sort")
    np.testing.assert_array_equal(Rs, oracle.sort(R, 0))
    Ss = oracle.sort(S, 0)

    A, B = Rs[:4000].copy(), Rs[4000:].copy()
    bA, bB = Block(0, 3, len(A)), Block(0, 3, len(B))
    merged = np.empty_like(Rs)
    _lib.check(lib.smj_merge(ctypes.byref(bA), p(A), ctypes.byref(bB), p(B), 0, p(merged)), "smj_merge")
    np.testing.assert_array_equal(merged, oracle.merge(A, B, 0))

    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    res = ctypes.c_void_p()
    rows = ctypes.c_int64(0)
    _lib.check(lib.smj_join(ctypes.byref(bR), p(Rs), ctypes.byref(bS), p(Ss), 0, 0, ctypes.byref(res),
                            ctypes.byref(rows)), "smj_join")
    got = np.ctypeslib.as_array(ctypes.cast(res, ctypes.POINTER(ctypes.c_int64)), shape=(rows.value * 4,)).copy()
    libc.free(res)
    np.testing.assert_array_equal(got.reshape(-1, 4), oracle.join(Rs, Ss, 0, 0))

    res = ctypes.c_void_p()
    _lib.check(lib.smj_sort_merge_join(ctypes.byref(bR), p(R), ctypes.byref(bS), p(S), 0, 100, 0, 200, 0, 0,
                                       ctypes.byref(res), ctypes.byref(rows), None), "smj_sort_merge_join")
    got = np.ctypeslib.as_array(ctypes.cast(res, ctypes.POINTER(ctypes.c_int64)), shape=(rows.value * 4,)).copy()
    libc.free(res)
    ref = oracle.join(oracle.select_sort(R, 0, 0, 100), oracle.select_sort(S, 0, 0, 200))
    np.testing.assert_array_equal(got.reshape(-1, 4), ref)
    # error behaviour mirrors DPU_ASSERT's inputs: invalid descriptor -> SMJ_ERR_INVALID
    bad = Block(0, 3, -1)
    assert lib.smj_sort(ctypes.byref(bad), p(R), 0) == -1
    assert lib.smj_sort(ctypes.byref(bR), p(R), 7) == -1


def test_c2_1m_pipeline_matches_oracle(gpu, oracle_built):
    """BASELINE config C2 (1M x 1M, uniform keys in [1, 3n], seeds 1/2)."""
    from smj import ops
    n = 1_000_000
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    got = ops.join(ops.select_sort(R, 0, 0, 5000), ops.select_sort(S, 0, 0, 5000))
    ref = oracle.join(oracle.select_sort(oracle.gen_uniform(n, 0, 1, 3 * n), 0, 0, 5000),
                      oracle.select_sort(oracle.gen_uniform(n, 0, 2, 3 * n), 0, 0, 5000))
    np.testing.assert_array_equal(host(got), ref)


@pytest.mark.parametrize("n,kind", [(100_000_000, "uniform"), (30_000_000, "zipf")])
def test_baseline_size_parity(gpu, oracle_built, n, kind):
    """C3 (1e8 x 1e8, the bench workload) and a Zipf(0.9) pair, bit for bit:
    the select+sort output against numpy's stable argsort of the selected
    input, and the join against the C oracle's zip join (O(n)) of those
    verified sorted tables.  (torch boolean-mask indexing is avoided as a
    checker: on this ROCm build it returns wrong rows above ~1e8 rows.)"""
    from smj import ops
    if kind == "uniform":
        R = ops.gen_uniform(n, seed=1, key_range=3 * n)
        S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    else:
        R = ops.gen_zipf(n, seed=3, domain=n, theta=0.9)
        S = ops.gen_zipf(n, seed=4, domain=n, theta=0.9)
    sorted_np = []
    for T in (R, S):
        got = host(ops.select_sort(T, 0, 0, 5000))
        t = host(T)
        keep = t[t[:, 0] > 5000]
        np.testing.assert_array_equal(got, keep[np.argsort(keep[:, 0], kind="stable")])
        sorted_np.append(got)
    Rs, Ss = (dev(a) for a in sorted_np)
    J = host(ops.join(Rs, Ss))
    np.testing.assert_array_equal(J, oracle.join(sorted_np[0], sorted_np[1]))


@pytest.mark.parametrize("binary,ktype", [("smj_app_u64", 1), ("smj_app_f64", 2)])
@pytest.mark.parametrize("case", ["test_10k", "atoi_edge", "neg_wide", "dup_heavy_sel", "wide12", "wide20_9"])
def test_smj_app_typed_result_csv(gpu, oracle_built, manifest, golden_dir, tmp_path, binary, ktype, case):
    """The app.c drop-in built with common.h T = uint64_t / double: result.csv
    byte-identical to cpu_app.c's pipeline restated with the same T (atoi
    values converted to T, '%ld' of (long) T on output; the reference's own
    '%ld' of a double is undefined behaviour, the restatement's cast is the
    contract)."""
    e = manifest["cases"][case]
    sel, keys = case_config(e, manifest["user_h_defaults"])
    out, ref = str(tmp_path / "result.csv"), str(tmp_path / "ref.csv")
    ins = [fixture_path(golden_dir, f) for f in e["inputs"]]
    cmd = [os.path.join(PKG, "bin", binary), *ins, "-o", out, "--select", *map(str, sel), "--keys", *map(str, keys)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=120)
    oracle.pipeline_csv(ins[0], ins[1], ref, sel, keys, ktype=ktype)
    assert sha(out) == sha(ref), case


@pytest.mark.parametrize("n,cols", [(0, 2), (1, 1), (4097, 2), (1_000_003, 3), (65_536, 9)])
def test_digest_matches_oracle(gpu, oracle_built, n, cols):
    """smj_dev_digest (bench.py's distributed self-check) against its C
    restatement, whole and in slices at their global positions."""
    from smj import ops
    rng = np.random.default_rng(7 * n + cols)
    t = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=(n, cols), dtype=np.int64, endpoint=True)
    d = dev(t).reshape(n, cols)
    assert ops.digest(d) == oracle.digest(t)
    a, b = n // 4, n // 2
    assert ops.digest(d[a:b], a) == oracle.digest(t[a:b], a)
    assert (ops.digest(d[:a]) + ops.digest(d[a:], a)) % (1 << 64) == oracle.digest(t)


@pytest.mark.gpu
@pytest.mark.parametrize("kc", [0, 1])
def test_packed_exchange_rows(gpu, oracle_built, kc):
    """The packed exchange format (smj.h smj_dev_partition_regions_pk /
    smj_dev_unpack_rows / smj_dev_sort_merge_join_begin_pk): the packed
    partition unpacks to the plain partition's rows exactly (keys on both
    sides of the base, negative payloads, a WHERE), a row whose payload does
    not fit int32 raises flag bit 2, and the pipeline on packed tables equals
    the pipeline on the plain ones (sorted rows and joined rows)."""
    import numpy as np
    from smj import ops
    from smj import dist as sdist
    rng = np.random.default_rng(17 + kc)
    n = 300_000
    def table(pay_hi):
        t = np.empty((n, 2), dtype=np.int64)
        t[:, kc] = rng.integers(-(1 << 40), 1 << 40, n) // (1 << 10) + (1 << 40)
        t[:, 1 - kc] = rng.integers(-pay_hi, pay_hi, n)
        return t
    R, S = table(1 << 30), table(1 << 31)
    dR, dS = torch.from_numpy(R).cuda(), torch.from_numpy(S).cuda()
    kb = int(np.median(R[:, kc]))
    bounds = sorted(set(int(x) for x in np.quantile(R[:, kc], [0.2, 0.5, 0.8]).astype(np.int64)))
    reg, _ = ops.region_capacities(R[:: 97, kc], n, bounds)
    for sel in (None, 0):
        c0 = torch.empty(len(bounds) + 2, dtype=torch.int64, device="cuda")
        c1 = torch.empty_like(c0)
        a = ops.partition_regions(dR, bounds, reg, c0, kc, kc, sel)
        b = ops.partition_regions(dR, bounds, reg, c1, kc, kc, sel, pack=(kb, 7))
        torch.cuda.synchronize()
        assert int(c1[-1]) == 0 and torch.equal(c0, c1)
        nb = len(bounds) + 1
        for q in range(nb):
            st, cnt = reg[q], int(c0[q])
            np.testing.assert_array_equal(ops.unpack_rows(b[st: st + cnt], kc, (kb, 7)).cpu().numpy(),
                                          a[st: st + cnt].cpu().numpy())
    # a payload that does not fit: flag bit 2
    c2 = torch.empty(len(bounds) + 2, dtype=torch.int64, device="cuda")
    dW = dR.clone()
    dW[123, 1 - kc] = 1 << 40
    ops.partition_regions(dW, bounds, reg, c2, kc, kc, None, pack=(kb, 0))
    torch.cuda.synchronize()
    assert int(c2[-1]) & 4
    # the pipeline on packed input (both, either) = on plain input
    pR = ops.partition_regions(dR, [], [0, n], torch.empty(2, dtype=torch.int64, device="cuda"), kc, pack=(kb, -5))
    pS = ops.partition_regions(dS, [], [0, n], torch.empty(2, dtype=torch.int64, device="cuda"), kc, pack=(kb + 99, 0))
    ref = ops.sort_merge_join(dR, dS, kc, kc, None, None)
    for p1, p2 in (((kb, -5), (kb + 99, 0)), (None, (kb + 99, 0)), ((kb, -5), None)):
        job = ops.sort_merge_join_begin_pk(pR[:n] if p1 else dR, pS[:n] if p2 else dS, kc, kc, p1, p2)
        got = job.end()
        for g, r in zip(got, ref):
            assert torch.equal(g, r)
    del sdist
