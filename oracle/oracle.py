"""Python handle on the CPU oracle (oracle/cpu_ref.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / the CPU baseline.  Every function
restates sort-merge-join/cpu_app.c (see cpu_ref.c for the line map); parity
of the restatement itself is pinned by tests/golden/ (outputs of the real
cpu_app.c, see tests/golden/make_goldens.py).
"""
import ctypes
import os
import subprocess  # noqa: F401 (build)

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libsmj_oracle.so")
# the restatement compiled with common.h T = uint64_t / double (key types 1, 2)
TYPED_LIBS = {1: os.path.join(HERE, "build", "libsmj_oracle_u64.so"),
              2: os.path.join(HERE, "build", "libsmj_oracle_f64.so")}
REF_LIB_U64 = os.path.join(HERE, "_ref", "libcpu_app_ref_u64.so")  # the real cpu_app.c, T = uint64_t
MT_LIB = os.path.join(HERE, "build", "libsmj_oracle_mt.so")  # multi-core port (cpu_mt.cpp), CPU baseline
CLI = os.path.join(HERE, "build", "cpu_ref")
REF_LIB = os.path.join(HERE, "_ref", "libcpu_app_ref.so")   # the real cpu_app.c (when built)
REF_DRIVER = os.path.join(HERE, "_ref", "ref_driver")

_lib = None
_typed = {}
_P = ctypes.c_void_p
_L = ctypes.c_int64
_TV = {0: ctypes.c_int64, 1: ctypes.c_uint64, 2: ctypes.c_double}  # C type of a T value


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(ktype=0):
    """The restatement for T = int64 (0), uint64 (1) or double (2)."""
    global _lib
    if ktype:
        if ktype not in _typed:
            if not os.path.exists(TYPED_LIBS[ktype]):
                build()
            _typed[ktype] = _bind(ctypes.CDLL(TYPED_LIBS[ktype]), ktype)
        return _typed[ktype]
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = _bind(ctypes.CDLL(LIB), 0)
    return _lib


def _bind(l, ktype):
    V = _TV[ktype]
    l.smj_ref_select_into.restype = _L
    l.smj_ref_select_into.argtypes = [ctypes.c_int, _L, _P, ctypes.c_int, V, _P]
    l.smj_ref_insertion_sort.restype = None
    l.smj_ref_insertion_sort.argtypes = [ctypes.c_int, _L, ctypes.c_int, _P]
    l.smj_ref_stable_sort.restype = ctypes.c_int
    l.smj_ref_stable_sort.argtypes = [ctypes.c_int, _L, ctypes.c_int, _P]
    l.smj_ref_join_count.restype = _L
    l.smj_ref_join_count.argtypes = [ctypes.c_int, _L, _P, ctypes.c_int, _L, _P, ctypes.c_int, ctypes.c_int]
    l.smj_ref_join.restype = _L
    l.smj_ref_join.argtypes = [ctypes.c_int, _L, _P, ctypes.c_int, _L, _P, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(_P)]
    l.smj_ref_gen_uniform.restype = None
    l.smj_ref_gen_uniform.argtypes = [_P, _L, _L, ctypes.c_uint64, ctypes.c_uint64]
    l.smj_ref_gen_zipf.restype = None
    l.smj_ref_gen_zipf.argtypes = [_P, _L, _L, ctypes.c_uint64, _L, ctypes.c_double, ctypes.c_double]
    l.smj_ref_gen_wide.restype = None
    l.smj_ref_gen_wide.argtypes = [_P, _L, _L, ctypes.c_uint64, ctypes.c_uint64, _L]
    l.smj_ref_digest.restype = ctypes.c_uint64
    l.smj_ref_digest.argtypes = [_P, _L, ctypes.c_int, _L]
    l.smj_ref_csv_size.restype = ctypes.c_int
    l.smj_ref_csv_size.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    l.smj_ref_load_csv.restype = ctypes.c_int
    l.smj_ref_load_csv.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]
    l.smj_ref_save_csv.restype = ctypes.c_int
    l.smj_ref_save_csv.argtypes = [ctypes.c_char_p, ctypes.c_int, _L, _P]
    l.smj_ref_pipeline_csv.restype = _L
    l.smj_ref_pipeline_csv.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, V,
                                       ctypes.c_int, V, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_double)]
    return l


_libc = ctypes.CDLL(None)
_libc.free.argtypes = [_P]


def _c(a):
    a = np.ascontiguousarray(a, dtype=np.int64)
    return a, a.ctypes.data_as(_P)


def select(table, select_col, select_val):
    """cpu_app.c select_in_cpu (:81-112)."""
    t, p = _c(table)
    out = np.empty_like(t)
    m = lib().smj_ref_select_into(t.shape[1], t.shape[0], p, select_col, int(select_val), out.ctypes.data_as(_P))
    return out[:m].copy()


def sort(table, key_col=0, insertion=False):
    """cpu_app.c insertion_sort_in_cpu (:172-202); stable.  insertion=False
    runs the O(n log n) merge sort with the identical output order."""
    t, p = _c(table)
    t = t.copy()
    p = t.ctypes.data_as(_P)
    if insertion:
        lib().smj_ref_insertion_sort(t.shape[1], t.shape[0], key_col, p)
    else:
        if lib().smj_ref_stable_sort(t.shape[1], t.shape[0], key_col, p) != 0:
            raise MemoryError("oracle sort")
    return t


def select_sort(table, key_col=0, select_col=0, select_val=None):
    t = table if select_val is None else select(table, select_col, select_val)
    return sort(t, key_col)


def join(R, S, key1=0, key2=0):
    """cpu_app.c join_in_cpu (:204-266)."""
    r, pr = _c(R)
    s, ps = _c(S)
    out = _P()
    j = lib().smj_ref_join(r.shape[1], r.shape[0], pr, s.shape[1], s.shape[0], ps, key1, key2, ctypes.byref(out))
    if j < 0:
        raise MemoryError("oracle join")
    tc = r.shape[1] + s.shape[1] - 1
    res = np.ctypeslib.as_array(ctypes.cast(out, ctypes.POINTER(ctypes.c_int64)), shape=(max(j, 1) * tc,))
    res = res[: j * tc].reshape(j, tc).copy()
    _libc.free(out)
    return res


def merge(a, b, key_col=0):
    """Stable merge of sorted runs (ties: a first) == sort(concat(a, b))."""
    return sort(np.concatenate([np.asarray(a, dtype=np.int64), np.asarray(b, dtype=np.int64)]), key_col)


def gen_uniform(rows, row0=0, seed=1, key_range=None):
    if key_range is None:
        key_range = 3 * rows
    out = np.empty((rows, 2), dtype=np.int64)
    lib().smj_ref_gen_uniform(out.ctypes.data_as(_P), row0, rows, seed, key_range)
    return out


def gen_wide(rows, row0=0, seed=1, plant_seed=1, plant_rows=0):
    """C3-wide keys: full-range signed int64; plant_rows > 0
    plants R's keys (table plant_seed, plant_rows rows) in a random third of
    the rows (smj_ref_gen_wide)."""
    out = np.empty((rows, 2), dtype=np.int64)
    lib().smj_ref_gen_wide(out.ctypes.data_as(_P), row0, rows, seed, plant_seed, plant_rows)
    return out


def digest(table, pos0=0):
    """The checker's restatement of smj_dev_digest (include/smj.h): an
    order-sensitive sum of per-row hashes of (global position, cells)."""
    t = np.ascontiguousarray(table)
    if t.dtype.itemsize != 8 or t.ndim != 2:
        raise ValueError("digest: 2-D table of 8-byte cells")
    return int(lib().smj_ref_digest(t.ctypes.data_as(_P), t.shape[0], max(t.shape[1], 1), int(pos0)))


def digest_np(table, pos0=0):
    """The same digest in numpy (an independent restatement for the tests)."""
    t = np.ascontiguousarray(table).view(np.uint64)
    M = np.uint64

    def mix(x):
        x = x + M(0x9E3779B97F4A7C15)
        x = (x ^ (x >> M(30))) * M(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> M(27))) * M(0x94D049BB133111EB)
        return x ^ (x >> M(31))

    with np.errstate(over="ignore"):
        h = mix(np.arange(pos0, pos0 + t.shape[0], dtype=np.int64).view(np.uint64) ^ M(0x5851F42D4C957F2D))
        for c in range(t.shape[1]):
            h = mix(h + t[:, c])
        return int(h.sum(dtype=np.uint64))


def zipf_zeta(n, theta):
    """sum_{i<=n} i^-theta: exact for i <= 1e6, Euler-Maclaurin for the tail
    (as smj_zipf_zeta)."""
    H = min(n, 1_000_000)
    z = float(np.sum(np.arange(H, 0, -1, dtype=np.float64) ** -theta))
    if n > H:
        a, b, s = float(H), float(n), 1.0 - theta
        z += (b ** s - a ** s) / s + 0.5 * (b ** -theta - a ** -theta) - theta / 12.0 * (b ** (-theta - 1) - a ** (-theta - 1))
    return z


def gen_zipf(rows, row0=0, seed=3, domain=100_000_000, theta=0.9, zeta=None):
    """Zipf(theta) keys over [1, domain], payload = global row (the device
    generator's restatement, smj_ref_gen_zipf)."""
    out = np.empty((rows, 2), dtype=np.int64)
    z = zipf_zeta(domain, theta) if zeta is None else zeta
    lib().smj_ref_gen_zipf(out.ctypes.data_as(_P), row0, rows, seed, domain, theta, z)
    return out


def load_csv(path):
    """cpu_app.c set_csv_size + load_csv (:15-79)."""
    c, r = ctypes.c_int(0), ctypes.c_int(0)
    if lib().smj_ref_csv_size(path.encode(), ctypes.byref(c), ctypes.byref(r)) != 0:
        raise FileNotFoundError(path)
    out = _P()
    lib().smj_ref_load_csv(path.encode(), c.value, r.value, ctypes.byref(out))
    n = c.value * r.value
    arr = np.ctypeslib.as_array(ctypes.cast(out, ctypes.POINTER(ctypes.c_int64)), shape=(max(n, 1),))
    res = arr[:n].reshape(r.value, c.value).copy()
    _libc.free(out)
    return res


def save_csv(path, table):
    t, p = _c(table)
    if t.ndim != 2:
        raise ValueError("2-D table expected")
    if lib().smj_ref_save_csv(path.encode(), t.shape[1], t.shape[0], p) != 0:
        raise OSError(path)


def time_cpu_pipeline(R, S, sel=(0, 5000, 0, 5000), keys=(0, 0)):
    """Time cpu_app.c's select -> insertion sort -> join (:336-344) on two
    in-memory tables, single thread.  Uses the REAL reference functions
    (oracle/_ref/libcpu_app_ref.so, built from /root/reference by
    `make -C oracle ref`) when present -> kind "reference"; otherwise our
    restatement -> kind "port".  Returns (seconds, joined_rows, kind)."""
    import time
    R = np.ascontiguousarray(R, dtype=np.int64)
    S = np.ascontiguousarray(S, dtype=np.int64)
    libc = ctypes.CDLL(None)
    libc.malloc.restype = _P
    libc.malloc.argtypes = [ctypes.c_size_t]

    def cbuf(a):
        p = libc.malloc(max(a.nbytes, 8))
        ctypes.memmove(p, a.ctypes.data, a.nbytes)
        return _P(p)

    if os.path.exists(REF_LIB):
        ref = ctypes.CDLL(REF_LIB)
        ref.select_in_cpu.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(_P), _L, _L]
        ref.insertion_sort_in_cpu.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]
        ref.join_in_cpu.argtypes = [ctypes.c_int, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P, ctypes.c_int,
                                    ctypes.c_int]
        a, b = cbuf(R), cbuf(S)
        ra, rb = ctypes.c_int(R.shape[0]), ctypes.c_int(S.shape[0])
        t0 = time.perf_counter()
        ref.select_in_cpu(R.shape[1], ctypes.byref(ra), ctypes.byref(a), sel[0], sel[1])
        ref.select_in_cpu(S.shape[1], ctypes.byref(rb), ctypes.byref(b), sel[2], sel[3])
        ref.insertion_sort_in_cpu(R.shape[1], ra.value, keys[0], ctypes.byref(a))
        ref.insertion_sort_in_cpu(S.shape[1], rb.value, keys[1], ctypes.byref(b))
        ref.join_in_cpu(R.shape[1], ra.value, a, S.shape[1], rb.value, b, keys[0], keys[1])
        dt = time.perf_counter() - t0
        rows = ctypes.c_int.in_dll(ref, "result_row_num").value
        res = _P.in_dll(ref, "result")
        for p in (a, b, res):
            _libc.free(p)
        res.value = None
        return dt, rows, "reference"
    t0 = time.perf_counter()
    Rs = select(R, sel[0], sel[1])
    Ss = select(S, sel[2], sel[3])
    Rs = sort(Rs, keys[0], insertion=True)
    Ss = sort(Ss, keys[1], insertion=True)
    rows = lib().smj_ref_join_count(Rs.shape[1], Rs.shape[0], Rs.ctypes.data_as(_P), Ss.shape[1], Ss.shape[0],
                                    Ss.ctypes.data_as(_P), keys[0], keys[1])
    j = join(Rs, Ss, keys[0], keys[1])
    dt = time.perf_counter() - t0
    assert len(j) == rows
    return dt, rows, "port"


def pipeline_csv(path1, path2, out_path, sel=(0, 5000, 0, 5000), keys=(0, 0), insertion=False, ktype=0):
    """cpu_app.c main (:303-361) with save_to_csv enabled; returns (rows, ms).
    ktype 1 / 2: the restatement compiled with T = uint64_t / double."""
    ms = ctypes.c_double(0)
    j = lib(ktype).smj_ref_pipeline_csv(path1.encode(), path2.encode(), out_path.encode() if out_path else None,
                                        sel[0], sel[1], sel[2], sel[3], keys[0], keys[1], int(insertion),
                                        ctypes.byref(ms))
    if j < 0:
        raise OSError("oracle pipeline failed")
    return j, ms.value


# ---- T = UINT64 / DOUBLE (common.h:3-9) --------------------------------------
def select_sort_t(table, ktype, key_col=0, select_col=0, select_val=None):
    """select + stable sort with T = uint64 (ktype 1) / double (2): table is an
    8-byte array of that dtype (or its int64 bits); returns the same dtype."""
    dt = {1: np.uint64, 2: np.float64}[ktype]
    t = np.ascontiguousarray(table).view(dt)
    if select_val is not None:
        out = np.empty_like(t)
        m = lib(ktype).smj_ref_select_into(t.shape[1], t.shape[0], t.ctypes.data_as(_P), select_col,
                                           _TV[ktype](select_val), out.ctypes.data_as(_P))
        t = out[:m].copy()
    else:
        t = t.copy()
    if lib(ktype).smj_ref_stable_sort(t.shape[1], t.shape[0], key_col, t.ctypes.data_as(_P)) != 0:
        raise MemoryError("oracle sort")
    return t


def join_t(R, S, ktype, key1=0, key2=0):
    """cpu_app.c join_in_cpu (:204-266) with T = uint64 / double."""
    dt = {1: np.uint64, 2: np.float64}[ktype]
    r = np.ascontiguousarray(R).view(dt)
    s = np.ascontiguousarray(S).view(dt)
    out = _P()
    j = lib(ktype).smj_ref_join(r.shape[1], r.shape[0], r.ctypes.data_as(_P), s.shape[1], s.shape[0],
                                s.ctypes.data_as(_P), key1, key2, ctypes.byref(out))
    if j < 0:
        raise MemoryError("oracle join")
    tc = r.shape[1] + s.shape[1] - 1
    res = np.ctypeslib.as_array(ctypes.cast(out, ctypes.POINTER(ctypes.c_int64)), shape=(max(j, 1) * tc,))
    res = res[: j * tc].reshape(j, tc).copy().view(dt)
    _libc.free(out)
    return res


# ---- multi-core port (cpu_mt.cpp): the CPU baseline at full size ----------------
_mt = None


def mt_pipeline(R, S, sel=(0, 5000, 0, 5000), keys=(0, 0), threads=16, outputs=False):
    """cpu_app.c's select -> stable sort -> zip join on `threads` cores
    (cpu_mt.cpp).  Returns (seconds, (m_R, m_S, J)) and, with outputs=True,
    the sorted tables and joined rows too."""
    global _mt
    if _mt is None:
        if not os.path.exists(MT_LIB):
            build()
        _mt = ctypes.CDLL(MT_LIB)
        _mt.smj_mt_pipeline.restype = ctypes.c_int
        _mt.smj_mt_pipeline.argtypes = [_P, _L, ctypes.c_int, _P, _L, ctypes.c_int] + \
            [ctypes.c_int, ctypes.c_int, _L] * 2 + [ctypes.c_int] * 3 + [_P, _P, _P, _P, _P]
    R = np.ascontiguousarray(R, dtype=np.int64)
    S = np.ascontiguousarray(S, dtype=np.int64)
    Rs, Ss = np.empty_like(R), np.empty_like(S)
    tc = R.shape[1] + S.shape[1] - 1
    out = np.empty((max(min(len(R), len(S)), 1), tc), dtype=np.int64) if outputs else None
    rows = (ctypes.c_int64 * 3)()
    secs = ctypes.c_double()
    sc1, sv1, sc2, sv2 = sel
    rc = _mt.smj_mt_pipeline(R.ctypes.data_as(_P), R.shape[0], R.shape[1], S.ctypes.data_as(_P), S.shape[0],
                             S.shape[1], int(sv1 is not None), sc1, int(sv1 or 0), int(sv2 is not None), sc2,
                             int(sv2 or 0), keys[0], keys[1], threads, Rs.ctypes.data_as(_P),
                             Ss.ctypes.data_as(_P), out.ctypes.data_as(_P) if outputs else None, rows,
                             ctypes.byref(secs))
    if rc != 0:
        raise ValueError("mt pipeline arguments")
    r = (int(rows[0]), int(rows[1]), int(rows[2]))
    if outputs:
        return secs.value, r, (Rs[: r[0]], Ss[: r[1]], out[: r[2]])
    return secs.value, r
