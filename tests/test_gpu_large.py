"""GPU parity of the partitioned mode (tables over 2^28 rows; BASELINE C4 and
C5 on one MI355X) of smj_dev_sort_merge_join.

* At small sizes the mode is forced (smj_debug_force_parts) and the outputs
  are compared with the CPU oracle bit for bit.
* At full size (C5: 1e8 x 1e9 Zipf(0.9); C4: 1e9 x 1e9 uniform) the outputs
  are checked through size-independent properties:
    - sorted tables: row count = the WHERE count, keys non-decreasing,
      payloads (= input row ids) strictly increasing within equal keys, and
      every output row equal to the input row its payload names -- together
      exactly "the stable sort of the selected rows";
    - joined rows: equal to a torch restatement of cpu_app.c's zip join
      (:204-266) over the verified sorted tables: R position i with key k
      pairs with S position lbS(k) + (i - lbR(k)) while that is < ubS(k);
    - key windows (the heaviest key, and a ~1e6-row window) of the INPUT
      tables, in input order, through the C oracle: sort and join are per-key
      operations, so the window's oracle result must equal the output slices
      holding its keys.
"""
import os

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

from test_gpu_msd import dev, host, ref_pipeline, table  # noqa: E402

SEL = 5000
CHUNK = 100_000_000


@pytest.fixture
def parts():
    from smj import ops
    yield ops.force_parts
    ops.force_parts(0)


FORCED = [
    # nr, ns, c1, c2, key1, key2, kind, select1, select2, parts
    (100_000, 100_000, 2, 2, 0, 0, "uniform", (0, 5000), (0, 5000), 2),
    (300_000, 200_000, 2, 2, 0, 0, "uniform", (0, 5000), (0, 5000), 7),
    (250_000, 250_000, 2, 2, 0, 0, "zipf", None, None, 8),
    (200_000, 150_000, 4, 5, 2, 4, "dom3", None, None, 5),
    (70_000, 9_000, 3, 2, 1, 0, "dups", (2, -10), None, 3),
    (120_000, 80_000, 2, 2, 0, 0, "extremes", None, None, 4),
    (300_000, 300_000, 2, 2, 0, 0, "same", None, None, 6),
    (40_000, 60_000, 8, 8, 7, 0, "wide", (0, 0), None, 16),
    (100_000, 100_000, 2, 2, 0, 0, "uniform", (0, 299_995), (0, 299_995), 4),
    (0, 50_000, 2, 2, 0, 0, "uniform", None, None, 3),
]


@pytest.mark.parametrize("nr,ns,c1,c2,k1,k2,kind,s1,s2,p", FORCED)
def test_partitioned_mode_matches_oracle(gpu, oracle_built, parts, nr, ns, c1, c2, k1, k2, kind, s1, s2, p):
    from smj import ops
    parts(p)
    rng = np.random.default_rng(nr * 3 + ns + p)
    R = table(rng, nr, c1, kind, k1, 0)
    S = table(rng, ns, c2, kind, k2, 10 ** 9)
    gR, gS, gJ = ops.sort_merge_join(dev(R).reshape(nr, c1), dev(S).reshape(ns, c2), k1, k2, s1, s2)
    Rs, Ss, J = ref_pipeline(R, S, k1, k2, s1, s2)
    np.testing.assert_array_equal(host(gR), Rs.reshape(-1, c1))
    np.testing.assert_array_equal(host(gS), Ss.reshape(-1, c2))
    if nr and ns:
        np.testing.assert_array_equal(host(gJ), J.reshape(-1, c1 + c2 - 1))


@pytest.mark.parametrize("kind,p", [("uniform", 5), ("zipf", 7), ("sorted", 4)])
def test_partition_fallback_when_a_region_overflows(gpu, oracle_built, parts, monkeypatch, kind, p):
    """The one-pass partition's part regions are sized from the key sample; a
    part over its region sends the call to the counting partition.  Regions
    scaled down to 30 % force that, and the result stays bit-exact."""
    from smj import ops
    parts(p)
    monkeypatch.setenv("SMJ_PART1_CAP", "0.3")
    rng = np.random.default_rng(p)
    base = "uniform" if kind == "sorted" else kind
    R = table(rng, 200_000, 2, base, 0, 0)
    S = table(rng, 150_000, 2, base, 0, 10 ** 9)
    if kind == "sorted":
        R = np.ascontiguousarray(R[np.argsort(R[:, 0], kind="stable")])
    gR, gS, gJ = ops.sort_merge_join(dev(R), dev(S), 0, 0, (0, SEL), (0, SEL))
    Rs, Ss, J = ref_pipeline(R, S, 0, 0, (0, SEL), (0, SEL))
    np.testing.assert_array_equal(host(gR), Rs.reshape(-1, 2))
    np.testing.assert_array_equal(host(gS), Ss.reshape(-1, 2))
    np.testing.assert_array_equal(host(gJ), J.reshape(-1, 3))


def test_partitioned_sorted_input_matches_oracle(gpu, oracle_built, parts):
    """Input already in key order (each sampled cluster of 16 rows falls in one
    part): the one-pass partition's regions, or its fallback, stay exact."""
    from smj import ops
    parts(6)
    rng = np.random.default_rng(11)
    R = table(rng, 300_000, 2, "dups", 0, 0)
    S = table(rng, 250_000, 2, "dups", 0, 10 ** 9)
    R = np.ascontiguousarray(R[np.argsort(R[:, 0], kind="stable")])
    S = np.ascontiguousarray(S[np.argsort(-S[:, 0], kind="stable")])  # descending: the sort reverses it stably
    gR, gS, gJ = ops.sort_merge_join(dev(R), dev(S), 0, 0, (0, -10), None)
    Rs, Ss, J = ref_pipeline(R, S, 0, 0, (0, -10), None)
    np.testing.assert_array_equal(host(gR), Rs.reshape(-1, 2))
    np.testing.assert_array_equal(host(gS), Ss.reshape(-1, 2))
    np.testing.assert_array_equal(host(gJ), J.reshape(-1, 3))


@pytest.mark.parametrize("case", [FORCED[1], FORCED[2], FORCED[3], FORCED[7], FORCED[4]])
def test_chunked_partition_matches_oracle(gpu, oracle_built, parts, monkeypatch, capfd, case):
    """The chunked one-pass partition (msd_part1c_kernel) with 3 chunks, so
    that every chunk walks many tiles and its parts span several sub-regions
    and partial part_a tiles: bit-exact, and the chunked path is the one taken."""
    from smj import ops
    nr, ns, c1, c2, k1, k2, kind, s1, s2, p = case
    parts(p)
    monkeypatch.setenv("SMJ_P1C_GRID", "3")
    monkeypatch.setenv("SMJ_DEBUG_PART1", "1")
    rng = np.random.default_rng(nr + 5 * ns + p)
    R = table(rng, nr, c1, kind, k1, 0)
    S = table(rng, ns, c2, kind, k2, 10 ** 9)
    gR, gS, gJ = ops.sort_merge_join(dev(R).reshape(nr, c1), dev(S).reshape(ns, c2), k1, k2, s1, s2)
    torch.cuda.synchronize()
    assert "chunked one-pass" in capfd.readouterr().err
    Rs, Ss, J = ref_pipeline(R, S, k1, k2, s1, s2)
    np.testing.assert_array_equal(host(gR), Rs.reshape(-1, c1))
    np.testing.assert_array_equal(host(gS), Ss.reshape(-1, c2))
    np.testing.assert_array_equal(host(gJ), J.reshape(-1, c1 + c2 - 1))


def test_chunked_partition_overflow_falls_back(gpu, oracle_built, parts, monkeypatch, capfd):
    """Input clustered by key (sorted R): every chunk's rows fall in a few
    parts, its sub-regions overflow, and the call takes the look-back
    partition instead -- still bit-exact."""
    from smj import ops
    parts(5)
    monkeypatch.setenv("SMJ_P1C_GRID", "4")
    monkeypatch.setenv("SMJ_DEBUG_PART1", "1")
    rng = np.random.default_rng(23)
    R = table(rng, 300_000, 2, "uniform", 0, 0)
    S = table(rng, 200_000, 2, "uniform", 0, 10 ** 9)
    R = np.ascontiguousarray(R[np.argsort(R[:, 0], kind="stable")])
    gR, gS, gJ = ops.sort_merge_join(dev(R), dev(S), 0, 0, (0, SEL), (0, SEL))
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    assert "chunked partition overflowed" in err and "one-pass regions" in err
    Rs, Ss, J = ref_pipeline(R, S, 0, 0, (0, SEL), (0, SEL))
    np.testing.assert_array_equal(host(gR), Rs.reshape(-1, 2))
    np.testing.assert_array_equal(host(gS), Ss.reshape(-1, 2))
    np.testing.assert_array_equal(host(gJ), J.reshape(-1, 3))


def test_partitioned_select_sort_matches_oracle(gpu, oracle_built, parts):
    from smj import ops
    parts(5)
    rng = np.random.default_rng(7)
    t = table(rng, 400_000, 3, "dups", 1, 0)
    got = ops.select_sort(dev(t), 1, 2, -20)
    np.testing.assert_array_equal(host(got), oracle.select_sort(t, 1, 2, -20).reshape(-1, 3))


# ---- full-size properties ----------------------------------------------------
def check_sorted_selection(T, got, sel):
    """got == the stable sort on column 0 of T's rows with column 0 > sel
    (column 1 of T = the row id)."""
    n = T.shape[0]
    want = 0
    for a in range(0, n, CHUNK):
        want += int((T[a: a + CHUNK, 0] > sel).sum())
    assert got.shape[0] == want
    m = got.shape[0]
    for a in range(0, m, CHUNK):
        b = min(m, a + CHUNK + 1)
        k, pay = got[a:b, 0], got[a:b, 1]
        assert bool((k > sel).all())
        dk = k[1:] - k[:-1]
        assert bool((dk >= 0).all()), "keys out of order"
        eq = dk == 0
        assert bool((pay[1:][eq] > pay[:-1][eq]).all()), "equal keys out of input order"
        assert torch.equal(T[got[a:b, 1]], got[a:b]), "an output row is not its input row"


def check_join(gR, gS, gJ):
    """gJ == the zip join of the (verified) sorted tables, restated in torch."""
    kR = gR[:, 0].contiguous()
    kS = gS[:, 0].contiguous()
    off = 0
    for a in range(0, kR.shape[0], CHUNK):
        k = kR[a: a + CHUNK]
        lbR = torch.searchsorted(kR, k, side="left")
        occ = torch.arange(a, a + k.shape[0], device=k.device) - lbR
        lbS = torch.searchsorted(kS, k, side="left")
        ubS = torch.searchsorted(kS, k, side="right")
        hit = occ < (ubS - lbS)
        part = (lbS + occ)[hit]
        want = torch.stack([gR[a: a + CHUNK, 0][hit], gR[a: a + CHUNK, 1][hit], gS[part, 1]], 1)
        assert torch.equal(gJ[off: off + want.shape[0]], want), f"joined rows differ in R chunk at {a}"
        off += want.shape[0]
        del lbR, occ, lbS, ubS, hit, part, want
    assert off == gJ.shape[0]


def check_window(R, S, gR, gS, gJ, lo, hi, sel=SEL):
    """Input rows with lo <= key <= hi (input order) through the C oracle ==
    the output slices holding those keys."""
    def window_in(T):
        m = (T[:, 0] >= lo) & (T[:, 0] <= hi)
        return host(T[m])

    def window_out(G):
        k = G[:, 0].contiguous()
        a = int(torch.searchsorted(k, torch.tensor([lo], device=k.device), side="left"))
        b = int(torch.searchsorted(k, torch.tensor([hi], device=k.device), side="right"))
        return host(G[a:b])

    Rw, Sw = window_in(R), window_in(S)
    Rs, Ss, J = ref_pipeline(Rw, Sw, 0, 0, (0, sel), (0, sel))
    np.testing.assert_array_equal(window_out(gR), Rs)
    np.testing.assert_array_equal(window_out(gS), Ss)
    np.testing.assert_array_equal(window_out(gJ), J)
    return len(Rs) + len(Ss), len(J)


def run_full(R, S, sel=SEL):
    from smj import ops
    gR, gS, gJ = ops.sort_merge_join(R, S, 0, 0, (0, sel), (0, sel))
    torch.cuda.synchronize()
    return gR, gS, gJ


def test_c5_full_size_one_gpu(gpu, oracle_built):
    """BASELINE C5 at full size on one MI355X: |R| = 1e8, |S| = 1e9,
    Zipf(0.9) keys over 1e8 values (seeds 3 / 4), WHERE col0 > 5000."""
    from smj import ops
    R = ops.gen_zipf(100_000_000, seed=3, domain=100_000_000, theta=0.9)
    S = ops.gen_zipf(1_000_000_000, seed=4, domain=100_000_000, theta=0.9)
    gR, gS, gJ = run_full(R, S)
    check_sorted_selection(R, gR, SEL)
    check_sorted_selection(S, gS, SEL)
    check_join(gR, gS, gJ)
    # the heaviest key (single-key groups far over the LDS capacity) and a window
    top = int(torch.mode(S[:1_000_000, 0]).values)
    rows, j = check_window(R, S, gR, gS, gJ, top, top)
    assert rows > 1_000_000 and j > 0
    mid = gS.shape[0] // 2
    check_window(R, S, gR, gS, gJ, int(gS[mid, 0]), int(gS[mid + 500_000, 0]))


C3W_SEL = -(1 << 63)  # WHERE col0 > INT64_MIN: ~every row passes


def test_c3_wide_full_size(gpu, oracle_built):
    """SURVEY 8(d)'s C3-wide stress input at full size: |R| = |S| = 1e8,
    full-range signed int64 keys (smj_dev_gen_wide), S planted with R's keys
    in a random third of its rows.  No group fits the narrow-span tiers
    (spans of ~2^45 keys per pass-B sub-bucket), so every group takes the
    wide-key path; packed pass-B rows are off (keys span 2^64)."""
    from smj import ops
    n = 100_000_000
    R = ops.gen_wide(n, seed=1)
    S = ops.gen_wide(n, seed=2, plant_seed=1, plant_rows=n)
    gR, gS, gJ = run_full(R, S, C3W_SEL)
    groups = ops.msd_groups()
    assert ops.msd_packb() == 0
    check_sorted_selection(R, gR, C3W_SEL)
    check_sorted_selection(S, gS, C3W_SEL)
    check_join(gR, gS, gJ)
    # ~n (1 - e^(-1/3)) distinct planted R rows (R's keys are distinct w.h.p.)
    assert 0.27 * n < gJ.shape[0] < 0.30 * n, gJ.shape[0]
    for q in (n // 7, n // 2):
        lo = int(gR[q, 0])
        hi = int(gR[q + 400_000, 0])
        rows, j = check_window(R, S, gR, gS, gJ, lo, hi, C3W_SEL)
        assert rows > 600_000 and j > 50_000
    # the extremes of the key range, where signed order matters
    check_window(R, S, gR, gS, gJ, -(1 << 63) + 1, int(gR[200_000, 0]), C3W_SEL)
    check_window(R, S, gR, gS, gJ, int(gR[n - 200_000, 0]), (1 << 63) - 1, C3W_SEL)
    print("c3-wide groups (dense, radix-tier, wide-tier, in-LDS LSD):", groups)


def test_c4_full_size_one_gpu(gpu, oracle_built):
    """BASELINE C4's tables (1e9 x 1e9, keys iid uniform in [1, 3e9], seeds
    1 / 2, WHERE col0 > 5000) on ONE MI355X through the partitioned mode."""
    from smj import ops
    n = 1_000_000_000
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    gR, gS, gJ = run_full(R, S)
    check_sorted_selection(R, gR, SEL)
    check_sorted_selection(S, gS, SEL)
    check_join(gR, gS, gJ)
    assert gJ.shape[0] > 0.2 * n
    lo = int(gR[n // 3, 0])
    rows, j = check_window(R, S, gR, gS, gJ, lo, lo + 1_500_000)
    assert rows > 500_000 and j > 0
    # the library's scratch (part regions, two per-part sets: ~100 GB here) goes
    # back to the device without smj_finalize, with the results still alive
    # 
    ops.trim()
    assert ops.scratch_bytes() == 0
    torch.cuda.empty_cache()
    big = torch.empty(100 * 2 ** 30, dtype=torch.uint8, device=R.device)
    del big


@pytest.mark.parametrize("workload,stages", [("c3", 1), ("c5", 2), ("c4", 3)])
def test_loopback_full_size_equals_single_call(gpu, workload, stages):
    """The distributed path at BASELINE sizes on one GPU (RCCL loopback,
    tools/loop_check.py): C3 with one stage sends 1.6 GB per table, C5 ~7 GB
    of S per stage, C4 5-9 GB per table and stage -- messages past RCCL's
    ~1 GiB point-to-point limit (profiles/r04/r04f/rccl_big.txt), so this
    exercises the piece cutting of smj/dist.py (before it, the C4 loopback
    join had 999,910,439 rows instead of 247,122,870).  The joined rows of
    every step equal the single call's bit for bit (the single call is
    oracle-checked at these sizes above and in test_gpu_msd.py)."""
    import subprocess
    import sys
    from smj import _lib
    _lib.load().smj_finalize()  # this process's scratch (the C4 test's ~50 GB) back to the device
    torch.cuda.empty_cache()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SMJ_DIST_STAGES=str(stages))
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "loop_check.py"), "--workload", workload,
                        "--steps", "2"], env=env, capture_output=True, text=True, timeout=600)
    wait_for_released_memory()
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def wait_for_released_memory(slack_gib=8, limit_s=120):
    """A child process's device memory is returned by the driver some time
    after the process exits (r06t: 265 GB still held when the next test
    allocated; SMJ_TEST_MEMLOG=1 in conftest.py shows it): wait until the
    memory held outside this process's library and torch is back under
    slack_gib, so that the next test starts with the device free."""
    import time
    from smj import ops
    t0 = time.time()
    while True:
        free, total = torch.cuda.mem_get_info()
        other = total - free - ops.scratch_bytes() - torch.cuda.memory_reserved()
        if other < slack_gib * 2 ** 30 or time.time() - t0 > limit_s:
            return
        time.sleep(0.5)


def test_repeated_partitioned_calls_agree(gpu):
    """Partitioned-mode calls of different sizes in one process, in both the
    overlapped (two parts in flight) and the profiled (parts in turn) order --
    the sequence bench.py's C4 loopback verification makes -- each equal to a
    fresh repetition of itself by the order-sensitive digest of all three
    outputs (r05f-r05j: a racy staged-kernel change showed up here as a wrong
    join count and inconsistent run metadata, tools/seq_sizes.py)."""
    from smj import _lib, ops
    _lib.load().smj_finalize()  # the earlier tests' scratch back to the device (this test reuses its own)
    torch.cuda.empty_cache()
    ref = {}
    for n, prof in ((292_000_000, False), (559_000_000, False), (292_000_000, True), (559_000_000, True),
                    (559_000_000, True)):
        R = ops.gen_uniform(n, seed=1, key_range=3 * n)
        S = ops.gen_uniform(n, seed=2, key_range=3 * n)
        ops.prof_enable(prof)
        try:
            gR, gS, gJ = ops.sort_merge_join(R, S, 0, 0, (0, SEL), (0, SEL))
            torch.cuda.synchronize()
        finally:
            ops.prof_enable(False)
            ops.prof_report()
        d = (gR.shape[0], gS.shape[0], gJ.shape[0], ops.digest(gR), ops.digest(gS), ops.digest(gJ))
        if n not in ref:  # the first call of each size against the property checks, not only itself
            check_sorted_selection(R, gR, SEL)
            check_sorted_selection(S, gS, SEL)
            check_join(gR, gS, gJ)
        assert ref.setdefault(n, d) == d, (n, prof, ref[n], d)
        del R, S, gR, gS, gJ
        torch.cuda.empty_cache()
