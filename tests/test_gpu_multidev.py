"""The sharded host-pointer path (smj_init(n > 1) / smj_init_devices): one
host thread per device of the set, range partition + exchange + the fused
pipeline per device (csrc/smj_host.hip), replacing app.c's spread of rows
over NR_DPUS (app.c:155-218) and its host-mediated merge tree.

On the one-GPU test box the set is n "virtual devices" that all map to GPU 0
(smj_init_devices with a repeated id): the exchange then runs as device
copies instead of xGMI peer copies, everything else is the multi-device
code.  Results must be byte-identical to the oracle for n = 1, 2, 4 and 8.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

import oracle
from conftest import case_config, fixture_path

pytestmark = pytest.mark.gpu

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd")


class Block(ctypes.Structure):
    _fields_ = [("table_num", ctypes.c_int), ("col_num", ctypes.c_int), ("row_num", ctypes.c_int)]


class Timing(ctypes.Structure):
    _fields_ = [("cpu_gpu_ms", ctypes.c_double), ("gpu_ms", ctypes.c_double), ("gpu_cpu_ms", ctypes.c_double)]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


@pytest.fixture
def lib(gpu):
    lib = gpu
    yield lib
    assert lib.smj_init(1) == 1  # leave the default single-device set for the other tests


def init_virtual(lib, n):
    ids = (ctypes.c_int * n)(*([0] * n))
    assert lib.smj_init_devices(ids, n) == n
    assert lib.smj_device_count() == n


def run_smj(lib, R, S, sel, keys, key_type=0):
    from smj import _lib
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    bR, bS = Block(0, R.shape[1], len(R)), Block(1, S.shape[1], len(S))
    res, rows, tm = ctypes.c_void_p(), ctypes.c_int64(0), Timing()
    m64 = (1 << 64) - 1
    _lib.check(lib.smj_sort_merge_join_typed(key_type, ctypes.byref(bR), _p(R), ctypes.byref(bS), _p(S), sel[0],
                                             sel[1] & m64, sel[2], sel[3] & m64, keys[0], keys[1], ctypes.byref(res),
                                             ctypes.byref(rows), ctypes.byref(tm)), "smj_sort_merge_join_typed")
    tc = R.shape[1] + S.shape[1] - 1
    got = np.ctypeslib.as_array(ctypes.cast(res, ctypes.POINTER(ctypes.c_int64)), shape=(max(rows.value, 1) * tc,))
    got = got[: rows.value * tc].copy().reshape(-1, tc)
    libc.free(res)
    assert tm.cpu_gpu_ms >= 0 and tm.gpu_ms > 0 and tm.gpu_cpu_ms >= 0
    return got


def tables(kind, nr, ns, rng):
    if kind == "uniform":
        R = np.stack([rng.integers(1, 3 * nr, nr), np.arange(nr)], 1)
        S = np.stack([rng.integers(1, 3 * nr, ns), 10 ** 9 + np.arange(ns)], 1)
    elif kind == "skew":  # one key holds most rows, negatives, 3 / 4 columns
        R = rng.integers(-500, 500, size=(nr, 3))
        S = rng.integers(-500, 500, size=(ns, 4))
        R[rng.random(nr) < 0.5, 1] = 17
        S[rng.random(ns) < 0.4, 2] = 17
        R[:, 0], S[:, 3] = np.arange(nr), -np.arange(ns)
    elif kind == "dups":
        R = rng.integers(0, 40, size=(nr, 2))
        S = rng.integers(0, 40, size=(ns, 2))
        R[:, 1], S[:, 1] = np.arange(nr), np.arange(ns)
    return np.ascontiguousarray(R, dtype=np.int64), np.ascontiguousarray(S, dtype=np.int64)


CASES = [
    # kind, nr, ns, (sc1, sv1, sc2, sv2), (k1, k2)
    ("uniform", 300_000, 250_000, (0, 5000, 0, 5000), (0, 0)),
    ("skew", 200_000, 150_000, (2, -400, 0, -1), (1, 2)),
    ("dups", 100_000, 120_000, (0, -1, 1, 50_000), (0, 0)),
    ("uniform", 7, 5, (0, 0, 0, 0), (0, 0)),
]


@pytest.mark.parametrize("kind,nr,ns,sel,keys", CASES)
def test_sharded_equals_oracle_for_every_device_count(lib, oracle_built, kind, nr, ns, sel, keys):
    rng = np.random.default_rng(nr + ns)
    R, S = tables(kind, nr, ns, rng)
    ref = oracle.join(oracle.select_sort(R, keys[0], sel[0], sel[1]), oracle.select_sort(S, keys[1], sel[2], sel[3]),
                      keys[0], keys[1])
    assert len(ref) > 0 or nr < 10
    for n in (1, 2, 4, 8):
        init_virtual(lib, n)
        got = run_smj(lib, R, S, sel, keys)
        np.testing.assert_array_equal(got, ref.reshape(-1, R.shape[1] + S.shape[1] - 1), err_msg=f"{n} devices")


def shard_rows(lib, n):
    out = (ctypes.c_int64 * n)()
    assert lib.smj_debug_shard_rows(out, n) == n
    return list(out)


@pytest.mark.parametrize("n_dev", [2, 4, 8])
def test_heavy_key_is_cut_by_occurrence(lib, oracle_built, n_dev):
    """A key holding 60 % of R and 50 % of S: the device set cuts it at an
    occurrence index (the same for R and S, so zip pairs stay together) and
    the devices' loads stay within 10 % of the mean (key-only splitters would
    put the whole key on one device: max / mean ~ 0.55 n_dev); the result is
    byte-identical to the oracle (smj/dist.py choose_cuts)."""
    rng = np.random.default_rng(21)
    nr, ns = 400_000, 300_000
    R = np.stack([rng.integers(-10_000, 10_000, nr), np.arange(nr)], 1)
    S = np.stack([rng.integers(-10_000, 10_000, ns), 10 ** 9 + np.arange(ns)], 1)
    R[rng.random(nr) < 0.6, 0] = 4242
    S[rng.random(ns) < 0.5, 0] = 4242
    R, S = np.ascontiguousarray(R, dtype=np.int64), np.ascontiguousarray(S, dtype=np.int64)
    sel = (1, -1, 0, -20_000)
    ref = oracle.join(oracle.select_sort(R, 0, 1, -1), oracle.select_sort(S, 0, 0, -20_000), 0, 0)
    init_virtual(lib, n_dev)
    np.testing.assert_array_equal(run_smj(lib, R, S, sel, (0, 0)), ref)
    rows = shard_rows(lib, n_dev)
    assert sum(rows) == nr + ns
    assert max(rows) / (sum(rows) / n_dev) <= 1.10, rows


def test_sharded_sort(lib, oracle_built):
    from smj import _lib
    rng = np.random.default_rng(3)
    R = np.ascontiguousarray(np.stack([rng.integers(-100, 100, 200_000), np.arange(200_000),
                                       rng.integers(0, 9, 200_000)], 1), dtype=np.int64)
    ref = oracle.sort(R, 0)
    for n in (2, 8):
        init_virtual(lib, n)
        got = R.copy()
        _lib.check(lib.smj_sort(ctypes.byref(Block(0, 3, len(R))), _p(got), 0), "smj_sort")
        np.testing.assert_array_equal(got, ref)


def test_sharded_typed_uint64(lib, oracle_built):
    """T = uint64: keys >= 2^63 sort after the others; the select compares
    unsigned too (oracle: the restatement built with -DUINT64)."""
    rng = np.random.default_rng(11)
    n = 150_000
    R = np.ascontiguousarray(np.stack([rng.integers(-1000, 1000, n), np.arange(n)], 1), dtype=np.int64)
    S = np.ascontiguousarray(np.stack([rng.integers(-1000, 1000, n), -np.arange(n)], 1), dtype=np.int64)
    sel = (0, 500, 0, (1 << 64) - 900)
    ref = oracle.join_t(oracle.select_sort_t(R, 1, 0, 0, 500), oracle.select_sort_t(S, 1, 0, 0, (1 << 64) - 900),
                        1, 0, 0)
    assert len(ref) > 0
    ref = np.ascontiguousarray(ref).view(np.int64)  # the same bits as the library's 8-byte cells
    for n_dev in (1, 4):
        init_virtual(lib, n_dev)
        np.testing.assert_array_equal(run_smj(lib, R, S, sel, (0, 0), key_type=1), ref)


def test_init_reports_the_real_device_set(lib):
    """smj_init returns the number of GPUs it really drives."""
    from smj import _lib  # noqa: F401
    import torch
    count = torch.cuda.device_count()
    assert lib.smj_init(0) == count and lib.smj_device_count() == count
    assert lib.smj_init(count + 5) == count
    bad = (ctypes.c_int * 2)(0, count + 3)
    assert lib.smj_init_devices(bad, 2) == -4  # SMJ_ERR_NODEVICE


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


@pytest.mark.parametrize("case", ["bundled_100k", "dup_heavy_sel", "wide_mixed", "atoi_edge"])
def test_smj_app_on_virtual_devices(gpu, manifest, golden_dir, tmp_path, case):
    """The app.c drop-in with a 4-entry device set (--devices 0,0,0,0):
    result.csv byte-identical to the reference cpu_app.c output."""
    e = manifest["cases"][case]
    sel, keys = case_config(e, manifest["user_h_defaults"])
    out = str(tmp_path / "result.csv")
    cmd = [os.path.join(PKG, "bin", "smj_app"), fixture_path(golden_dir, e["inputs"][0]),
           fixture_path(golden_dir, e["inputs"][1]), "-o", out, "--select", *map(str, sel), "--keys", *map(str, keys),
           "--devices", "0,0,0,0"]
    r = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=120)
    assert "on 4 GPU(s)" in r.stdout
    assert sha(out) == e["sha256"], case
