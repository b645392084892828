"""CPU checks of the drop-in boundary: libsmj_hip.so builds for gfx950, loads
without a GPU, and exports exactly what include/smj.h declares; the C host's
CSV layer (libsmj_csv.so) reproduces the reference ingest/egress bytes."""
import ctypes
import filecmp
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, REPO, fixture_path

import oracle

HEADER = os.path.join(REPO, "include", "smj.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", text)
    return sorted(set(re.findall(r"\b(smj_[a-z_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["smj_init", "smj_finalize", "smj_select", "smj_sort", "smj_merge", "smj_join",
                 "smj_sort_merge_join", "smj_dev_select_sort", "smj_dev_join", "smj_strerror"]:
        assert must in names


def test_library_exports_every_declared_symbol(pkg_built):
    lib = ctypes.CDLL(os.path.join(PKG, "lib", "libsmj_hip.so"))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_table_covers_header(pkg_built):
    from smj import _lib
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_library_is_gfx950_code_object(pkg_built):
    """The .hip_fatbin offload bundle carries exactly one device target: gfx950."""
    data = open(os.path.join(PKG, "lib", "libsmj_hip.so"), "rb").read()
    assert b"__CLANG_OFFLOAD_BUNDLE__" in data
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}


def test_no_device_is_reported_not_crashed(pkg_built):
    """Without a GPU the product path fails loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from smj import _lib
    lib = _lib.load(build_if_missing=False)
    assert lib.smj_init(1) == -4  # SMJ_ERR_NODEVICE
    assert lib.smj_strerror(-4) == b"no usable gfx950 device"


# ---- CSV layer of the C host (product code) against the oracle -------------
def csv_lib():
    lib = ctypes.CDLL(os.path.join(PKG, "lib", "libsmj_csv.so"))
    lib.smj_csv_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_void_p)]
    lib.smj_csv_save.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p]
    lib.smj_csv_set_threads.argtypes = [ctypes.c_int]
    return lib


@pytest.fixture(params=[1, 7], ids=["serial", "7threads"])
def csv_threads(request):
    """Both CSV code paths: the serial reference loop and the chunked parallel one."""
    lib = csv_lib()
    lib.smj_csv_set_threads(request.param)
    yield request.param
    lib.smj_csv_set_threads(0)


def load_with(lib, path):
    c, r, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_void_p()
    assert lib.smj_csv_load(str(path).encode(), ctypes.byref(c), ctypes.byref(r), ctypes.byref(p)) == 0
    n = c.value * r.value
    got = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int64)), shape=(max(n, 1),))[:n].copy()
    ctypes.CDLL(None).free(p)
    return got.reshape(r.value, c.value)


@pytest.mark.parametrize("name", ["data1.csv.gz", "data_1.csv.gz", "kat_r.csv", "kat_s.csv", "dup_r.csv",
                                  "atoi_r.csv", "atoi_s.csv", "wide_s.csv", "neg_r.csv", "empty_t.csv",
                                  "one_r.csv"])
def test_csv_load_matches_reference_semantics(pkg_built, oracle_built, golden_dir, name, csv_threads):
    lib = csv_lib()
    path = fixture_path(golden_dir, name)
    c, r, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_void_p()
    assert lib.smj_csv_load(path.encode(), ctypes.byref(c), ctypes.byref(r), ctypes.byref(p)) == 0
    n = c.value * r.value
    got = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int64)), shape=(max(n, 1),))[:n].copy()
    ctypes.CDLL(None).free(p)
    ref = oracle.load_csv(path)
    assert (r.value, c.value) == ref.shape
    np.testing.assert_array_equal(got.reshape(ref.shape), ref)


def test_csv_long_lines_and_nul(pkg_built, oracle_built, tmp_path, csv_threads):
    """fgets(1024) line splitting and C-string truncation at NUL, as the reference."""
    p = tmp_path / "odd.csv"
    long_tok = "7" * 1500
    p.write_bytes(b"a,b\n1,2\n" + long_tok.encode() + b",3\n4\x005,6\n" + b"9," * 600 + b"\n8,8")
    lib = csv_lib()
    c, r, ptr = ctypes.c_int(), ctypes.c_int(), ctypes.c_void_p()
    assert lib.smj_csv_load(str(p).encode(), ctypes.byref(c), ctypes.byref(r), ctypes.byref(ptr)) == 0
    n = c.value * r.value
    got = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_int64)), shape=(max(n, 1),))[:n].copy()
    ref = oracle.load_csv(str(p))
    assert (r.value, c.value) == ref.shape
    np.testing.assert_array_equal(got.reshape(ref.shape), ref)


def test_csv_save_bytes(pkg_built, oracle_built, tmp_path, csv_threads):
    rng = np.random.default_rng(1)
    t = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=(5000, 7), dtype=np.int64,
                     endpoint=True)
    t[0, :] = [0, -1, 1, np.iinfo(np.int64).min, np.iinfo(np.int64).max, 10, -10]
    a, b = str(tmp_path / "a.csv"), str(tmp_path / "b.csv")
    assert csv_lib().smj_csv_save(a.encode(), 7, len(t), t.ctypes.data) == 0
    oracle.save_csv(b, t)
    assert filecmp.cmp(a, b, shallow=False)


def test_csv_parallel_load_spills_and_odd_lines(pkg_built, oracle_built, tmp_path):
    """A messy file cut into many chunks: rows with extra tokens spill into
    the next rows' cells (the reference's unbounded token index), short rows,
    empty fields, CRLF, NUL, > 1023-byte lines, atoi overflow -- the parallel
    loader must equal the oracle (reference semantics) cell for cell."""
    rng = np.random.default_rng(5)
    lines = [b"k,v,w"]
    for i in range(60_000):
        kind = rng.integers(0, 12)
        if kind == 0:  # spill: 3..9 extra tokens
            lines.append(b",".join(str(int(x)).encode() for x in rng.integers(-99, 99, size=3 + rng.integers(1, 10))))
        elif kind == 1:  # short row
            lines.append(str(int(rng.integers(-5, 5))).encode())
        elif kind == 2:
            lines.append(b",,%d,,%d\r" % (i, -i))
        elif kind == 3:
            lines.append(b"%d,9\x00%d,1" % (i, i))
        elif kind == 4 and i % 50 == 0:  # a long line: fgets pieces
            lines.append(b"5," * 700 + b"1")
        elif kind == 5:
            lines.append(b" +%d, -%d,99999999999999999999" % (i, i))
        else:
            lines.append(b"%d,%d,%d" % (int(rng.integers(0, 10**6)), i, -i))
    p = tmp_path / "messy.csv"
    p.write_bytes(b"\n".join(lines) + b"\n")
    lib = csv_lib()
    ref = oracle.load_csv(str(p))
    for nt in (1, 3, 16, 61):
        lib.smj_csv_set_threads(nt)
        got = load_with(lib, p)
        assert got.shape == ref.shape, nt
        np.testing.assert_array_equal(got, ref, err_msg=f"{nt} threads")
    lib.smj_csv_set_threads(0)


def test_csv_parallel_save_equals_serial(pkg_built, tmp_path):
    rng = np.random.default_rng(9)
    t = rng.integers(-(10**12), 10**12, size=(700_001, 3), dtype=np.int64)
    lib = csv_lib()
    outs = []
    for nt in (1, 5):
        lib.smj_csv_set_threads(nt)
        path = str(tmp_path / f"o{nt}.csv")
        assert lib.smj_csv_save(path.encode(), 3, len(t), t.ctypes.data) == 0
        outs.append(path)
    lib.smj_csv_set_threads(0)
    assert filecmp.cmp(outs[0], outs[1], shallow=False)
