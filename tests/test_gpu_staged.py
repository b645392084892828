"""The staged host-pointer path: one-device
smj_sort_merge_join copies each table over PCIe in chunks of 3,440,640 rows
(smj_api.hip msd_staged_sort_merge_join) and runs part_a on every chunk as soon
as it lands.  These cases span several chunks with ragged last chunks, |R| !=
|S|, a WHERE that drops rows and non-default key / select columns, and compare
against the CPU oracle bit for bit -- once in this process (staged) and once in
a child process with SMJ_STAGED=0 (one copy per table, then the pipeline).
Reference: app.c:221-244 / 342-359 push the row slices, app.c:290-292 /
763-772 time the CPU-DPU / DPU / DPU-CPU buckets these calls report."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

CHUNK = 4 * 5 * 3 * 7 * 8192  # msd_staged_sort_merge_join's chunk: 3,440,640 rows

CASES = {
    # name: (nr, ns, c1, c2, key1, key2, (sel_col1, sel_val1), (sel_col2, sel_val2))
    "two_col": (8_000_123, 9_100_001, 2, 2, 0, 0, (0, 1_000_000), (1, 777)),
    "mixed_width": (7_300_001, 3 * CHUNK + 1, 3, 5, 2, 1, (1, 250), (4, -5)),
}


class Block(ctypes.Structure):
    _fields_ = [("table_num", ctypes.c_int), ("col_num", ctypes.c_int), ("row_num", ctypes.c_int)]


class Timing(ctypes.Structure):
    _fields_ = [("cpu_gpu_ms", ctypes.c_double), ("gpu_ms", ctypes.c_double), ("gpu_cpu_ms", ctypes.c_double)]


def make_tables(name):
    nr, ns, c1, c2, k1, k2, s1, s2 = CASES[name]
    rng = np.random.default_rng(nr ^ ns)
    R = rng.integers(1, 3 * nr, size=(nr, c1), dtype=np.int64)
    S = rng.integers(1, 3 * nr, size=(ns, c2), dtype=np.int64)
    if c1 > 2:  # select on a small-domain column: the WHERE drops ~half the rows
        R[:, 1] = rng.integers(0, 500, size=nr)
    if c2 > 2:
        S[:, 4] = rng.integers(-10, 10, size=ns)
    R[:, (k1 + 1) % c1] = np.arange(nr)  # payload = row id: stability is visible
    S[:, (k2 + 1) % c2] = 10 ** 12 + np.arange(ns)
    return R, S


def run_host_join(name, lib):
    """smj_sort_merge_join on host tables (as app.c would call it)."""
    nr, ns, c1, c2, k1, k2, s1, s2 = CASES[name]
    R, S = make_tables(name)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    res, rows, tm = ctypes.c_void_p(), ctypes.c_int64(0), Timing()
    rc = lib.smj_sort_merge_join(ctypes.byref(Block(0, c1, nr)), p(R), ctypes.byref(Block(1, c2, ns)), p(S),
                                 s1[0], s1[1], s2[0], s2[1], k1, k2, ctypes.byref(res), ctypes.byref(rows),
                                 ctypes.byref(tm))
    assert rc == 0, f"smj_sort_merge_join -> {rc}"
    tc = c1 + c2 - 1
    got = np.ctypeslib.as_array(ctypes.cast(res, ctypes.POINTER(ctypes.c_int64)),
                                shape=(rows.value * tc,)).copy().reshape(-1, tc)
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    libc.free(res)
    return got, (tm.cpu_gpu_ms, tm.gpu_ms, tm.gpu_cpu_ms)


def expected(name):
    nr, ns, c1, c2, k1, k2, s1, s2 = CASES[name]
    R, S = make_tables(name)
    return oracle.join(oracle.select_sort(R, k1, s1[0], s1[1]), oracle.select_sort(S, k2, s2[0], s2[1]), k1, k2)


@pytest.fixture(scope="module")
def lib1(gpu):
    from smj import _lib
    lib = _lib.load()
    assert lib.smj_init(1) >= 1
    return lib


@pytest.mark.parametrize("name", sorted(CASES))
def test_staged_multi_chunk_matches_oracle(lib1, oracle_built, monkeypatch, name):
    nr, ns = CASES[name][:2]
    assert max(nr, ns) > 2 * CHUNK and nr % CHUNK and ns % CHUNK  # several chunks, ragged last ones
    # the result's threaded D2H (smj_host.hip d2h_result: 8 parts, 8 MiB pinned
    # slots) from 1 MiB on, so that these results take it with ragged parts
    monkeypatch.setenv("SMJ_D2H_MIN", str(1 << 20))
    got, tm = run_host_join(name, lib1)
    ref = expected(name)
    assert len(ref) > 0
    np.testing.assert_array_equal(got, ref)
    assert all(t >= 0 for t in tm)


@pytest.mark.parametrize("name", sorted(CASES))
def test_serial_copy_path_matches_oracle(gpu, oracle_built, tmp_path, name):
    """SMJ_STAGED=0 is read once per process: run it in a child process."""
    out = str(tmp_path / "got.npy")
    here = os.path.dirname(os.path.abspath(__file__))
    code = (f"import sys; sys.path[:0] = {[here, PKG, os.path.join(REPO, 'oracle'), REPO]!r}\n"
            "import numpy as np\n"
            "from smj import _lib\n"
            "import test_gpu_staged as t\n"
            "lib = _lib.load(); assert lib.smj_init(1) >= 1\n"
            f"got, tm = t.run_host_join({name!r}, lib)\n"
            f"np.save({out!r}, got)\n")
    env = dict(os.environ, SMJ_STAGED="0")
    subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=240,
                   cwd=here)
    np.testing.assert_array_equal(np.load(out), expected(name))
