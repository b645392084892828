"""The multi-GPU driver (smj/dist.py) on CPU: world sizes 2 and 3 over gloo.

The HIP operators are replaced -- in this test only -- by an oracle-backed
stand-in with the same interface, so what is tested here is the distributed
orchestration: splitter choice, stable bucket scatter semantics, the
all_to_all exchange in source-rank order, the per-rank radix base, and that
concatenating rank outputs in rank order reproduces cpu_app.c's result.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle


class OracleOps:
    """CPU stand-in for smj.dist.HipOps (test infrastructure)."""

    @staticmethod
    def select_sort(table, key_col=0, select_col=0, select_val=None, key_base=0):
        t = table.numpy()
        out = oracle.select_sort(t, key_col, select_col, select_val)
        if len(out):  # the radix base must be a lower bound of every key
            biased = (out[:, key_col].astype(np.uint64) ^ np.uint64(1 << 63))
            assert int(biased.min()) >= key_base
        return torch.from_numpy(out.reshape(-1, t.shape[1]))

    @staticmethod
    def join(R, S, key1=0, key2=0):
        return torch.from_numpy(oracle.join(R.numpy(), S.numpy(), key1, key2).reshape(-1, R.shape[1] + S.shape[1] - 1))

    @staticmethod
    def sort_merge_join(R, S, key1=0, key2=0, select1=None, select2=None):
        Rs = OracleOps.select_sort(R, key1, *(select1 or (0, None)))
        Ss = OracleOps.select_sort(S, key2, *(select2 or (0, None)))
        return Rs, Ss, OracleOps.join(Rs, Ss, key1, key2)

    @staticmethod
    def _keep(T, key, sc, sv, spl):
        t = T.numpy()
        keep = t if sv is None else t[t[:, sc] > sv]
        bucket = np.searchsorted(spl.numpy(), keep[:, key], side="left")
        return keep, bucket

    @staticmethod
    def partition_count(T, spl, key=0, sc=0, sv=None):
        keep, bucket = OracleOps._keep(T, key, sc, sv, spl)
        counts = np.bincount(bucket, minlength=spl.numel() + 1).tolist()
        mm = (int(keep[:, key].min()), int(keep[:, key].max())) if len(keep) else ((1 << 63) - 1, -(1 << 63))
        return counts, mm

    @staticmethod
    def partition_scatter(T, spl, counts, key=0, sc=0, sv=None):
        keep, bucket = OracleOps._keep(T, key, sc, sv, spl)
        return torch.from_numpy(keep[np.argsort(bucket, kind="stable")].copy())

    @staticmethod
    def partition_plan(T, bounds, counts, key=0, sc=0, sv=None):
        keep, bucket = OracleOps._keep(T, key, sc, sv, torch.tensor(bounds, dtype=torch.int64))
        counts.copy_(torch.from_numpy(np.bincount(bucket, minlength=len(bounds) + 1).astype(np.int64)))
        return keep, bucket

    @staticmethod
    def partition_apply(T, bounds, plan, key=0, sc=0, sv=None):
        keep, bucket = plan
        return torch.from_numpy(keep[np.argsort(bucket, kind="stable")].copy())

    @staticmethod
    def region_capacities(own, n, bounds):
        from smj import ops as hip_ops  # pure host arithmetic (no GPU)
        return hip_ops.region_capacities(own, n, bounds)

    @staticmethod
    def partition_regions(T, bounds, reg, counts, key=0, sc=0, sv=None):
        """smj_dev_partition_regions' contract: bucket b's rows (stable) at
        reg[b], at most reg[nb + b] of them; exact counts; flag on overflow."""
        keep, bucket = OracleOps._keep(T, key, sc, sv, torch.tensor(bounds, dtype=torch.int64))
        nb = len(bounds) + 1
        out = np.zeros((max(max(reg[b] + reg[nb + b] for b in range(nb)), 1), T.shape[1]), dtype=np.int64)
        over = 0
        for b in range(nb):
            rows = keep[bucket == b]
            c = min(len(rows), reg[nb + b])
            out[reg[b]: reg[b] + c] = rows[:c]
            over |= len(rows) > reg[nb + b]
        cnt = np.bincount(bucket, minlength=nb).astype(np.int64)
        counts.copy_(torch.from_numpy(np.concatenate([cnt, [int(over)]]).astype(np.int64)))
        return torch.from_numpy(out)

    @staticmethod
    def partition(T, spl, key=0, sc=0, sv=None):
        counts, _ = OracleOps.partition_count(T, spl, key, sc, sv)
        return counts, OracleOps.partition_scatter(T, spl, counts, key, sc, sv)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, R, S, cfg, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "pim-sort-merge-join_amd"), os.path.join(repo, "oracle"), here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    backend = cfg.get("backend", "gloo")
    if backend == "nccl":  # RCCL: one rank per GPU, the only one here is cuda:0
        torch.cuda.set_device(rank)
    dist.init_process_group(backend, rank=rank, world_size=world)
    from smj import dist as sdist
    from test_dist_gloo import OracleOps as Ops
    # contiguous, uneven slices in input order
    cuts_r = np.linspace(0, len(R), world + 1).astype(int)
    cuts_s = np.sqrt(np.linspace(0, 1, world + 1)) * len(S)
    cuts_s = cuts_s.astype(int)
    r = torch.from_numpy(R[cuts_r[rank]:cuts_r[rank + 1]].copy())
    s = torch.from_numpy(S[cuts_s[rank]:cuts_s[rank + 1]].copy())
    ops = Ops
    if cfg.get("gpu"):  # the product operators (HipOps) on cuda:0, exchange staged through gloo
        torch.cuda.set_device(0)
        r, s, ops = r.cuda(), s.cuda(), None
    stats = {}
    out = sdist.sort_merge_join(r, s, select=cfg["select"], keys=cfg["keys"], ops=ops, samples=cfg["samples"],
                                stats=stats, stages=cfg.get("stages"), loopback=cfg.get("loopback"))
    np.save(os.path.join(outdir, f"rank{rank}.npy"), out.cpu().numpy())
    if rank == 0:
        np.save(os.path.join(outdir, "load.npy"), np.array([stats["load_max_over_mean"]]))
        with open(os.path.join(outdir, "stats.json"), "w") as f:
            json.dump({k: stats.get(k) for k in ("exchange_packed", "pack_fallbacks", "stages")}, f)
    dist.barrier()
    dist.destroy_process_group()


def make_tables(kind, n):
    rng = np.random.default_rng(42)
    if kind == "uniform":
        return oracle.gen_uniform(n, 0, 1, 3 * n), oracle.gen_uniform(n, 0, 2, 3 * n)
    if kind == "dups":  # heavy duplicates, 3 columns, key in column 1
        R = rng.integers(0, 40, size=(n, 3)).astype(np.int64)
        S = rng.integers(0, 40, size=(n // 2, 3)).astype(np.int64)
        R[:, 0], S[:, 2] = np.arange(n), np.arange(n // 2) + 10 ** 6
        return R, S
    if kind == "widepay":  # payloads over int32: the packed exchange falls back to plain rows
        R, S = oracle.gen_uniform(n, 0, 1, 3 * n), oracle.gen_uniform(n, 0, 2, 3 * n)
        R[:, 1] = rng.integers(-(1 << 62), 1 << 62, n)
        S[:, 1] = rng.integers(-(1 << 62), 1 << 62, n)
        return R, S
    if kind == "widekeys":  # full-range keys (C3-wide): the sample's span rules packing out up front
        R, S = oracle.gen_wide(n, 0, 1), oracle.gen_wide(n, 0, 2, 1, n)
        return R, S
    if kind == "skew":  # one key carries most rows, negative keys too
        R = rng.integers(-1000, 1000, size=(n, 2)).astype(np.int64)
        S = rng.integers(-1000, 1000, size=(n, 2)).astype(np.int64)
        R[rng.random(n) < 0.6, 0] = 17
        S[rng.random(n) < 0.5, 0] = 17
        R[:, 1], S[:, 1] = np.arange(n), -np.arange(n)
        return R, S
    if kind == "farout":  # dense keys, 1 % far outliers and the int64 extremes (round 6's stress shape)
        tabs = []
        for x in range(2):
            k = rng.integers(0, 10 ** 6, size=n, dtype=np.int64)
            m = rng.random(n) < 0.01
            k[m] = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=int(m.sum()), dtype=np.int64,
                                endpoint=True)
            k[rng.choice(n, 40, replace=False)] = np.iinfo(np.int64).min
            k[rng.choice(n, 30, replace=False)] = np.iinfo(np.int64).max
            tabs.append(np.stack([k, x * 10 ** 9 + np.arange(n, dtype=np.int64)], axis=1))
        return tabs[0], tabs[1]
    raise ValueError(kind)


@pytest.mark.parametrize("world,kind,cfg", [
    (2, "uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 64}),
    (3, "uniform", {"select": (0, 100, 0, 20000), "keys": (0, 0), "samples": 16}),
    (2, "dups", {"select": (2, 5, 0, 5), "keys": (1, 1), "samples": 32}),
    (3, "skew", {"select": (0, -900, 0, -2000), "keys": (0, 0), "samples": 8}),
    (2, "uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 64, "stages": 1}),
    (3, "skew", {"select": (0, -900, 0, -2000), "keys": (0, 0), "samples": 8, "stages": 1}),
    (4, "dups", {"select": (2, 5, 0, 5), "keys": (1, 1), "samples": 32, "stages": 8}),
    (8, "uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 64}),
])
def test_distributed_equals_single(tmp_path, oracle_built, world, kind, cfg):
    _run_and_check(tmp_path, world, kind, cfg, 30_000)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,cfg", [
    ("uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True}),
    ("dups", {"select": (2, 5, 0, 5), "keys": (1, 1), "samples": 256, "gpu": True}),
    ("skew", {"select": (0, -900, 0, -2000), "keys": (0, 0), "samples": 1024, "gpu": True}),
    ("uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True, "stages": 1}),
    ("farout", {"select": (0, -(1 << 63), 0, -(1 << 63)), "keys": (0, 0), "samples": 4096, "gpu": True}),
])
def test_distributed_hip_two_ranks_one_gpu(tmp_path, oracle_built, pkg_built, kind, cfg):
    """The product path of smj/dist.py -- HIP smj_dev_partition and the
    fused local smj_dev_sort_merge_join -- with 2 ranks sharing cuda:0 and the
    all_to_all staged through gloo (RCCL needs one GPU per rank)."""
    _run_and_check(tmp_path, 2, kind, cfg, 400_000)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,cfg", [
    ("uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True}),
    ("skew", {"select": (0, -900, 0, -2000), "keys": (0, 0), "samples": 1024, "gpu": True}),
])
def test_distributed_hip_eight_ranks_one_gpu(tmp_path, oracle_built, pkg_built, kind, cfg):
    """The bench's N = 8 configuration (8 ranks, the default stage count:
    W K - 1 = 31 splitters, 4 stages per rank) on the product operators, the
    8 ranks sharing cuda:0 and the exchange staged through gloo."""
    _run_and_check(tmp_path, 8, kind, cfg, 800_000)


def test_uneven_stage_shares(tmp_path, oracle_built, monkeypatch):
    """Stage shares within a rank (SMJ_DIST_STAGE_FRAC): segment boundaries at
    uneven cumulative fractions for the splitters and the cuts; the result is
    the same rows in the same order."""
    monkeypatch.setenv("SMJ_DIST_STAGE_FRAC", "1,3")
    _run_and_check(tmp_path, 3, "uniform", {"select": (0, 100, 0, 20000), "keys": (0, 0), "samples": 64,
                                             "stages": 2}, 30_000)


def test_choose_cuts_fractions():
    from smj import dist as sdist
    # 8 equal single-row buckets; boundaries at 1/4 and 1/2 -> cuts at buckets 2 and 4
    GR, GS = [1] * 8, [0] * 8
    assert sdist.choose_cuts(GR, GS, [False] * 8, 3, [0.25, 0.5]) == [(2, 0), (4, 0)]
    assert sdist.seg_fracs(2, 2, [1, 3]) == [0.125, 0.5, 0.625]


def test_region_overflow_falls_back(tmp_path, oracle_built, monkeypatch):
    """Regions sized below the bucket counts (SMJ_DIST_REGION_SCALE): the
    overflowing ranks re-partition with plan / apply and the result is the
    same (the one-read pass counts every row, so the cuts do not change)."""
    monkeypatch.setenv("SMJ_DIST_REGION_SCALE", "0.5")
    _run_and_check(tmp_path, 3, "skew", {"select": (0, -900, 0, -2000), "keys": (0, 0), "samples": 8}, 30_000)


@pytest.mark.parametrize("world", [1, 2])
def test_loopback_exchange_gloo(tmp_path, oracle_built, world):
    """Loopback mode (each rank's own segments through send / receive to
    itself; one rank takes the whole distributed path) gives the same result."""
    _run_and_check(tmp_path, world, "uniform",
                   {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 64, "loopback": True}, 30_000)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,cfg", [
    ("uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True}),
    ("skew", {"select": (0, -900, 0, -2000), "keys": (0, 0), "samples": 1024, "gpu": True, "stages": 4}),
    # messages cut into 64 KiB pieces (SMJ_DIST_MAX_MSG; RCCL corrupts p2p
    # messages over ~2 GiB, profiles/r04/r04e): hundreds of pieces per stage
    ("uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True, "max_msg": 65536}),
    # payloads over int32: packing falls back to plain rows on every rank
    ("widepay", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True, "expect_pack": (
        [False, False], 2)}),
    # full-range keys: not packed to begin with (no thrown-away packed partition)
    ("widekeys", {"select": (0, -(1 << 63), 0, -(1 << 63)), "keys": (0, 0), "samples": 4096, "gpu": True,
                  "expect_pack": ([False, False], 0)}),
    # dense keys with far outliers and the extremes (the final tiers' oversized groups, round 6)
    ("farout", {"select": (0, -(1 << 63), 0, -(1 << 63)), "keys": (0, 0), "samples": 4096, "gpu": True}),
    ("uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True, "expect_pack": (
        [True, True], 0)}),
    # the packed exchange turned off
    ("uniform", {"select": (0, 5000, 0, 5000), "keys": (0, 0), "samples": 4096, "gpu": True, "pack": "0"}),
])
def test_distributed_rccl_loopback_one_gpu(tmp_path, oracle_built, pkg_built, monkeypatch, kind, cfg):
    """The RCCL transport of smj/dist.py on the one GPU a test box has: one
    rank under the nccl backend (RCCL) in loopback mode, so the partition,
    the device-resident send buffers, the staged batch_isend_irecv over the
    RCCL communicator (to itself) and the stage-overlapped local pipeline
    all run as on the 8-GPU node, bit-exact against the oracle."""
    if cfg.get("max_msg"):
        monkeypatch.setenv("SMJ_DIST_MAX_MSG", str(cfg["max_msg"]))
    if cfg.get("pack"):
        monkeypatch.setenv("SMJ_DIST_PACK", cfg["pack"])
    _run_and_check(tmp_path, 1, kind, dict(cfg, backend="nccl", loopback=True), 1_000_000)
    if cfg.get("expect_pack"):
        st = json.loads((tmp_path / "stats.json").read_text())
        assert (st["exchange_packed"], st["pack_fallbacks"]) == tuple(cfg["expect_pack"]), st


def test_heavy_key_is_split_by_occurrence(tmp_path, oracle_built):
    """with 60 % of R and 50 % of S on one key, key-only
    splitters would put that key on one rank; (key, occurrence) cuts spread
    its occurrences (the same cut for R and S keeps the zip pairs together)
    and the rank loads stay within 10 % of the mean."""
    # (the cuts use R's exact counts and S's sample estimate -- R's first stage
    # leaves before S is counted -- so the sample must resolve the heavy key's
    # share of S: 512 samples per table and rank here, 4096 in production)
    load = _run_and_check(tmp_path, 4, "skew", {"select": (0, -900, 0, -2000), "keys": (0, 0), "samples": 512},
                          40_000)
    assert load < 1.10, load


@pytest.mark.parametrize("n", [1, 2, 4095, 4096, 4097, 16_777_217, 50_000_000, 100_000_000, 2_000_000_000])
def test_sample_index_stays_in_bounds(n):
    """The splitter sample's row indices are exact int64 (a float32
    linspace rounds n - 1 up to n above 2^24 rows)."""
    from smj import dist as sdist
    idx = sdist.sample_index(n, 4096)
    assert idx.dtype == torch.int64 and idx.numel() == min(n, 4096)
    assert int(idx.min()) == 0 and int(idx.max()) == n - 1
    assert bool((idx[1:] > idx[:-1]).all()) if idx.numel() > 1 else True


def test_stage_count():
    from smj import dist as sdist
    # 2 (W K - 1) boundaries must fit the 64-bucket partition kernel
    assert [sdist.stage_count(w, 4) for w in (2, 4, 8, 16)] == [4, 4, 4, 2]
    assert sdist.stage_count(8, 1) == 1 and sdist.stage_count(32, 4) == 1


def test_message_pieces_tile_the_range(monkeypatch):
    """A (peer, bucket range) message is cut into pieces of <= MAX_MSG_BYTES;
    sender and receiver cut identically (same lengths from their own base)."""
    from smj import dist as sdist
    monkeypatch.setattr(sdist, "MAX_MSG_BYTES", 1000)
    p = sdist._pieces(5, 5 + 200, 2)  # 62 rows of 16 B per piece
    assert p[0] == (5, 67) and p[-1][1] == 205 and all(b - a <= 62 for a, b in p)
    assert all(p[i][1] == p[i + 1][0] for i in range(len(p) - 1))
    q = sdist._pieces(1000, 1200, 2)
    assert [b - a for a, b in p] == [b - a for a, b in q]
    assert sdist._pieces(7, 7, 2) == []


def test_slice_ranges_match_slice_counts():
    """Per-segment (bucket, lo, hi) ranges: their sizes are slice_counts', they
    tile each bucket's local rows, and a single-key bucket is split at the
    occurrence cut."""
    from smj import dist as sdist
    local, prefix = [3, 0, 7, 5, 2], [1, 0, 4, 0, 9]
    cuts = [(2, 6), (2, 6), (3, 0), (4, 10)]
    rs = sdist.slice_ranges(local, prefix, cuts, 5)
    assert [sum(h - l for _, l, h in r) for r in rs] == sdist.slice_counts(local, prefix, cuts, 5)
    assert rs[0] == [(0, 0, 3), (2, 0, 2)] and rs[1] == [] and rs[2] == [(2, 2, 7)]
    assert rs[3] == [(3, 0, 5), (4, 0, 1)] and rs[4] == [(4, 1, 2)]


def test_choose_cuts_pure():
    from smj import dist as sdist
    s, single = sdist.bucket_bounds(torch.tensor([5, 17, 17, 17, 40]))
    assert s == [4, 5, 16, 17, 39, 40] and single == [False, True, False, True, False, True, False]
    # bucket 3 (key 17) holds 60 of 100 R rows and 30 of 60 S rows
    GR, GS = [10, 0, 10, 60, 10, 0, 10], [5, 0, 5, 30, 10, 0, 10]
    cuts = sdist.choose_cuts(GR, GS, single, 4)
    assert cuts[0][0] == 3 and cuts[1][0] == 3 and cuts == sorted(cuts)
    # every rank's share of R + S = 160 rows is within one occurrence pair of 40
    edges = [0]
    for b, o in cuts:
        edges.append(sum(GR[:b]) + sum(GS[:b]) + (min(o, GR[b]) + min(o, GS[b]) if b < len(GR) else 0))
    edges.append(160)
    assert all(abs((edges[i + 1] - edges[i]) - 40) <= 2 for i in range(4)), edges


def _run_and_check(tmp_path, world, kind, cfg, n):
    R, S = make_tables(kind, n)
    mp.spawn(_worker, args=(world, free_port(), R, S, cfg, str(tmp_path)), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    sc1, sv1, sc2, sv2 = cfg["select"]
    k1, k2 = cfg["keys"]
    ref = oracle.join(oracle.select_sort(R, k1, sc1, sv1), oracle.select_sort(S, k2, sc2, sv2), k1, k2)
    assert len(ref) > 0
    np.testing.assert_array_equal(got, ref)
    return float(np.load(tmp_path / "load.npy")[0])


def _splitter_worker(rank, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "pim-sort-merge-join_amd"), here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    from smj import dist as sdist
    from smj import ops
    bad = []
    rng = np.random.default_rng(5)
    cases = [(1_000_000, 700_000, 2, 2, 0, 0, 4096, 2, None), (1_000_000, 700_000, 2, 2, 0, 0, 4096, 3,
                                                               [0.05, 0.15]),
             (5000, 3, 3, 2, 1, 0, 64, 7, None), (0, 90_000, 2, 4, 0, 3, 1024, 4, [0.1, 0.5, 0.9]),
             (0, 0, 2, 2, 0, 0, 512, 3, None), (200_000, 200_000, 2, 2, 0, 0, 4096, 32, None)]
    for nr, ns, cr, cs, kr, ks, samples, parts, fracs in cases:
        R = torch.from_numpy(rng.integers(-50, 50, size=(nr, cr)).astype(np.int64)).cuda()
        S = torch.from_numpy(rng.integers(-(1 << 62), 1 << 62, size=(ns, cs)).astype(np.int64)).cuda()
        if ns:
            S[: ns // 3, ks] = 7  # a heavy key: repeated splitters
        res = []
        for o in (sdist.HipOps, None):
            own, est = [], {}
            spl = sdist.choose_splitters([(R, kr), (S, ks)], 1, None, samples, parts=parts, own=own, fracs=fracs,
                                         est=est, ops=o)
            res.append((spl, [np.asarray(x).tolist() for x in own], np.asarray(est["all"]).tolist()))
        if res[0] != res[1]:
            bad.append((nr, ns, parts, fracs))
    np.save(os.path.join(outdir, "bad.npy"), np.array([len(bad)]))
    with open(os.path.join(outdir, "bad.txt"), "w") as f:
        f.write(repr(bad))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_hip_splitters_equal_torch_path(tmp_path, pkg_built):
    """smj_dev_dist_sample + smj_dev_dist_splitters (the RCCL path's splitter
    choice: one sample kernel, one all_gather_into_tensor, one order-statistic
    kernel, one host copy) give the torch path's splitters, own samples and
    gathered estimate exactly: even and stage-fraction positions, a repeated
    (heavy) key, empty tables, 3 / 4-column rows, up to 32 parts."""
    mp.spawn(_splitter_worker, args=(free_port(), str(tmp_path)), nprocs=1, join=True)
    assert int(np.load(tmp_path / "bad.npy")[0]) == 0, (tmp_path / "bad.txt").read_text()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 3, 8])
def test_dist_splitters_kernel_many_ranks(pkg_built, world):
    """smj_dev_dist_splitters on a gathered buffer of `world` ranks (as the
    all_gather lays it out: per rank a 5-word header, R's then S's sampled
    keys, INT64_MAX pads) against numpy: the keys at sorted positions
    max(0, (q + 1) L / parts - 1) -- and at the stage-fraction positions --
    with ranks of different valid counts, duplicates and INT64 extremes."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
    from smj import ops
    rng = np.random.default_rng(world)
    samples = 1024
    H, stride = 5, 5 + 2 * samples
    for trial in range(4):
        allb = np.full((world, stride), np.iinfo(np.int64).max, dtype=np.int64)
        for r in range(world):
            c0, c1 = int(rng.integers(0, samples + 1)), int(rng.integers(0, samples + 1))
            if trial == 3:
                c0 = c1 = 0  # no samples anywhere: every splitter 0
            allb[r, :H] = [c0 + c1, c0, c1, 10 * c0, 10 * c1]
            keys = rng.integers(-1000, 1000, c0 + c1) * (1 << 50) if trial else rng.integers(-5, 5, c0 + c1)
            if c0 + c1 > 2:
                keys[0], keys[1] = np.iinfo(np.int64).min, np.iinfo(np.int64).max
            allb[r, H: H + c0 + c1] = keys
        L = int(allb[:, 0].sum())
        srt = np.sort(allb[:, H:].reshape(-1))
        for parts, fr in ((world * 2, None), (min(32, world * 4), "q")):
            q20 = None
            if fr:
                cum = np.sort(rng.random(parts - 1))
                q20 = [int(round(f * (1 << 20))) for f in cum]
                pos = [max(0, q * L // (1 << 20) - 1) for q in q20]
            else:
                pos = [max(0, i * L // parts - 1) for i in range(1, parts)]
            ref = [0] * (parts - 1) if L == 0 else [int(srt[p]) for p in pos]
            out = ops.dist_splitters(torch.from_numpy(allb.reshape(-1)).cuda(), world, stride, parts, q20)
            got = out.cpu().numpy()
            assert got[:parts - 1].tolist() == ref and int(got[parts - 1]) == L, (trial, parts, fr)


def test_key_base_and_stage_defaults():
    """The packed exchange's key base is the middle of the gathered key
    sample of the table (all ranks; 0 without samples, exact in int64 at the
    extremes), and one rank runs one stage only while its tables fit one
    pipeline call."""
    from smj import dist as sdist
    I64 = np.iinfo(np.int64)
    H, cap = 5, 8
    a = np.full((2, H + cap), I64.max, dtype=np.int64)
    a[0, :H] = [3, 2, 1, 10, 10]
    a[0, H:H + 3] = [-7, 5, 100]       # R: -7, 5; S: 100
    a[1, :H] = [2, 1, 1, 10, 10]
    a[1, H:H + 2] = [40, -300]         # R: 40; S: -300
    est = {"all": a, "H": H, "nt": 2}
    assert sdist._key_base(est, 0) == (-7 + 40) // 2
    assert sdist._key_base(est, 1) == (-300 + 100) // 2
    b = a.copy()
    b[:, 1:3] = 0
    assert sdist._key_base({"all": b, "H": H, "nt": 2}, 0) == 0
    c = a.copy()
    c[0, H] = I64.min
    c[1, H] = I64.max - 1
    assert sdist._key_base({"all": c, "H": H, "nt": 2}, 0) == (int(I64.min) + int(I64.max) - 1) // 2
    if sdist.DEFAULT_STAGES is None:
        assert sdist.default_stages(1, 100_000_000) == 1
        assert sdist.default_stages(1, 1_000_000_000) == 3
        assert sdist.default_stages(8, 10) == 4
