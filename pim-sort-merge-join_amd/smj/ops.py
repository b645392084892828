"""Device-resident operators of the sort-merge-join hot path (torch tensors in,
torch tensors out; the work is done by the HIP kernels behind libsmj_hip.so).

Tables are 2-D int64 CUDA tensors [rows, cols], row-major and contiguous --
the reference's T[row_num * col_num] layout (common.h).  Names follow the
reference pipeline (cpu_app.c / app.c): select, sort, merge, join.
"""
import ctypes
import json

import torch

from . import _lib

BIAS = 1 << 63


def biased(key: int) -> int:
    """The unsigned radix order of a signed key: key ^ 2^63 (as uint64)."""
    return (int(key) + BIAS) & ((1 << 64) - 1)


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else ctypes.c_void_p(0)


def _table(t, name):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.int64 and t.dim() == 2
            and t.is_contiguous()):
        raise ValueError(f"{name} must be a contiguous 2-D int64 CUDA tensor")
    return t


def _out(t, name, rows, cols, like, dtype=torch.int64):
    """A caller-provided output buffer: the C layer trusts its capacity, so an
    undersized, strided or foreign buffer is refused here."""
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == dtype and t.dim() == 2 and t.is_contiguous()):
        raise ValueError(f"{name} must be a contiguous 2-D {dtype} CUDA tensor")
    if t.device != like.device:
        raise ValueError(f"{name} is on {t.device}, the inputs on {like.device}")
    if t.shape[1] != cols or t.shape[0] < rows:
        raise ValueError(f"{name} has shape {tuple(t.shape)}, needs at least ({rows}, {cols})")
    return t


def select_sort(table, key_col=0, select_col=0, select_val=None, key_base=0, out=None, stream=None):
    """out[:m] <- stable sort on table[:, key_col] of the rows with
    table[:, select_col] > select_val (all rows when select_val is None).
    Returns the view out[:m] (m is read back: the call synchronises once)."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    out = torch.empty_like(table) if out is None else _out(out, "out", n, cols, table)
    m = ctypes.c_int64(0)
    use = select_val is not None
    _lib.check(lib.smj_dev_select_sort(_ptr(table), n, cols, int(use), select_col,
                                       int(select_val) if use else 0, key_col, biased_base(key_base),
                                       _ptr(out), ctypes.byref(m), _stream(stream)), "smj_dev_select_sort")
    return out[: m.value]


def select_sort_lsd(table, key_col=0, select_col=0, select_val=None, key_base=0, out=None, stream=None):
    """select_sort on the LSD radix path (the MSD pipeline's fallback)."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    out = torch.empty_like(table) if out is None else _out(out, "out", n, cols, table)
    m = ctypes.c_int64(0)
    use = select_val is not None
    _lib.check(lib.smj_dev_select_sort_lsd(_ptr(table), n, cols, int(use), select_col,
                                           int(select_val) if use else 0, key_col, biased_base(key_base),
                                           _ptr(out), ctypes.byref(m), _stream(stream)), "smj_dev_select_sort_lsd")
    return out[: m.value]


KEY_INT64, KEY_UINT64, KEY_DOUBLE = 0, 1, 2  # smj.h SMJ_KEY_* (common.h T)


def _bits(v, key_type):
    """64-bit pattern of a select value of type T."""
    import struct
    if key_type == KEY_DOUBLE:
        return struct.unpack("<Q", struct.pack("<d", float(v)))[0]
    return int(v) & ((1 << 64) - 1)


def sort_merge_join(R, S, key1=0, key2=0, select1=None, select2=None, R_sorted=None, S_sorted=None, out=None,
                    stream=None, key_type=KEY_INT64):
    """The fused hot path (cpu_app.c main :303-364): select (select = (col, val)
    keeps rows with row[col] > val; None keeps all), stable sort on the key,
    1:1 zip join.  Returns (R_sorted[:mR], S_sorted[:mS], out[:J]).
    key_type KEY_UINT64 / KEY_DOUBLE compares keys and select values as
    common.h's T = uint64_t / double (tables: int64 tensors holding the bits,
    or float64 tensors for double)."""
    lib = _lib.load()
    if key_type != KEY_INT64:
        return _sort_merge_join_typed(lib, R, S, key1, key2, select1, select2, R_sorted, S_sorted, out, stream,
                                      key_type)
    _table(R, "R")
    _table(S, "S")
    nr, c1 = R.shape
    ns, c2 = S.shape
    if S.device != R.device:
        raise ValueError("R and S must be on the same device")
    R_sorted = torch.empty_like(R) if R_sorted is None else _out(R_sorted, "R_sorted", nr, c1, R)
    S_sorted = torch.empty_like(S) if S_sorted is None else _out(S_sorted, "S_sorted", ns, c2, R)
    if out is None:
        out = torch.empty((max(min(nr, ns), 1), c1 + c2 - 1), dtype=torch.int64, device=R.device)
    else:
        _out(out, "out", min(nr, ns), c1 + c2 - 1, R)
    rows = (ctypes.c_int64 * 3)()
    s1 = select1 or (0, 0)
    s2 = select2 or (0, 0)
    _lib.check(lib.smj_dev_sort_merge_join(_ptr(R), nr, c1, int(select1 is not None), s1[0], int(s1[1]), key1,
                                           _ptr(S), ns, c2, int(select2 is not None), s2[0], int(s2[1]), key2,
                                           _ptr(R_sorted), _ptr(S_sorted), _ptr(out), rows, _stream(stream)),
               "smj_dev_sort_merge_join")
    return R_sorted[: rows[0]], S_sorted[: rows[1]], out[: rows[2]]


class SortMergeJoinJob:
    """sort_merge_join in two halves (smj_dev_sort_merge_join_begin / _end):
    the pipeline is enqueued by sort_merge_join_begin, and end(out) compacts
    the joined rows into out (allocated if None), waits and returns what
    sort_merge_join returns.  Until end() the thread must not start another
    pipeline call; the tables and the job must stay alive."""

    def __init__(self, lib, handle, R, S, R_sorted, S_sorted, stream, shapes=None):
        self._lib, self._h = lib, handle
        self._keep = (R, S)
        self.R_sorted, self.S_sorted, self._stream = R_sorted, S_sorted, stream
        # (rows, columns) of R and S as tables (packed inputs hold one word per row)
        self._shapes = shapes or (tuple(R.shape), tuple(S.shape))

    def end(self, out=None):
        """Finish the job.  The C job is released whatever happens here: an
        unusable `out` still ends it (the C call drains the stream and frees
        the thread's pipeline) before the error is raised."""
        if self._h is None:
            raise RuntimeError("job already ended")
        R, S = self._keep
        (nr, c1), (ns, c2) = self._shapes
        h, self._h = self._h, None
        rows = (ctypes.c_int64 * 3)()
        try:
            if out is None:
                out = torch.empty((max(min(nr, ns), 1), c1 + c2 - 1), dtype=torch.int64, device=R.device)
            else:
                _out(out, "out", min(nr, ns), c1 + c2 - 1, R)
        except BaseException:
            self._lib.smj_dev_sort_merge_join_end(h, None, rows)  # returns SMJ_ERR_INVALID, job released
            self._keep = None
            raise
        rc = self._lib.smj_dev_sort_merge_join_end(h, _ptr(out), rows)
        self._keep = None
        _lib.check(rc, "smj_dev_sort_merge_join_end")
        return self.R_sorted[: rows[0]], self.S_sorted[: rows[1]], out[: rows[2]]

    def abandon(self):
        """End a job whose result is not wanted (waits for its kernels)."""
        if self._h is not None:
            h, self._h = self._h, None
            self._lib.smj_dev_sort_merge_join_end(h, None, (ctypes.c_int64 * 3)())
            self._keep = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.abandon()  # a job not ended inside the block
        return False

    def __del__(self):
        # a job dropped without end() would keep its thread's pipeline scratch
        # (every later pipeline call on the thread returns SMJ_ERR_INVALID)
        try:
            self.abandon()
        except Exception:
            pass


def sort_merge_join_begin(R, S, key1=0, key2=0, select1=None, select2=None, R_sorted=None, S_sorted=None,
                          stream=None):
    """Enqueue sort_merge_join up to its sort/join kernel and return a
    SortMergeJoinJob at once (int64 tables); job.end(out) finishes it."""
    lib = _lib.load()
    _table(R, "R")
    _table(S, "S")
    nr, c1 = R.shape
    ns, c2 = S.shape
    if S.device != R.device:
        raise ValueError("R and S must be on the same device")
    R_sorted = torch.empty_like(R) if R_sorted is None else _out(R_sorted, "R_sorted", nr, c1, R)
    S_sorted = torch.empty_like(S) if S_sorted is None else _out(S_sorted, "S_sorted", ns, c2, R)
    s1 = select1 or (0, 0)
    s2 = select2 or (0, 0)
    h = ctypes.c_void_p()
    _lib.check(lib.smj_dev_sort_merge_join_begin(_ptr(R), nr, c1, int(select1 is not None), s1[0], int(s1[1]), key1,
                                                 _ptr(S), ns, c2, int(select2 is not None), s2[0], int(s2[1]), key2,
                                                 _ptr(R_sorted), _ptr(S_sorted), _stream(stream), ctypes.byref(h)),
               "smj_dev_sort_merge_join_begin")
    return SortMergeJoinJob(lib, h, R, S, R_sorted, S_sorted, stream)


def _packed_rows(t, name):
    if not (t.is_cuda and t.dtype == torch.int64 and t.is_contiguous() and (t.dim() == 1 or (t.dim() == 2 and
                                                                                            t.shape[1] == 1))):
        raise ValueError(f"{name} must be a contiguous int64 CUDA tensor of packed rows (n or n x 1)")
    return t.shape[0]


def sort_merge_join_begin_pk(R, S, key1=0, key2=0, pack1=None, pack2=None, R_sorted=None, S_sorted=None,
                             stream=None):
    """sort_merge_join_begin of two 2-column tables without a select, either
    of which may be packed (smj_dev_sort_merge_join_begin_pk): packX = None
    for an n x 2 table, or (key_base, other_base) for n packed words
    (partition_regions(..., pack=...)).  Packed tables over 1.6e8 rows raise
    (unpack_rows them first).  job.end(out) finishes it."""
    lib = _lib.load()
    shp = []
    for t, pk, name in ((R, pack1, "R"), (S, pack2, "S")):
        if pk is None:
            _table(t, name)
            if t.shape[1] != 2:
                raise ValueError(f"{name} must have 2 columns")
            shp.append((t.shape[0], 2))
        else:
            shp.append((_packed_rows(t, name), 2))
    (nr, _), (ns, _) = shp
    R_sorted = torch.empty((nr, 2), dtype=torch.int64, device=R.device) if R_sorted is None else \
        _out(R_sorted, "R_sorted", nr, 2, R)
    S_sorted = torch.empty((ns, 2), dtype=torch.int64, device=R.device) if S_sorted is None else \
        _out(S_sorted, "S_sorted", ns, 2, R)
    p1, p2 = pack1 or (0, 0), pack2 or (0, 0)
    h = ctypes.c_void_p()
    _lib.check(lib.smj_dev_sort_merge_join_begin_pk(_ptr(R), nr, key1, int(pack1 is not None), int(p1[0]), int(p1[1]),
                                                    _ptr(S), ns, key2, int(pack2 is not None), int(p2[0]), int(p2[1]),
                                                    _ptr(R_sorted), _ptr(S_sorted), _stream(stream), ctypes.byref(h)),
               "smj_dev_sort_merge_join_begin_pk")
    return SortMergeJoinJob(lib, h, R, S, R_sorted, S_sorted, stream, shapes=tuple(shp))


def unpack_rows(packed, key_col, pack, out=None, stream=None):
    """smj_dev_unpack_rows: n packed words -> an n x 2 table (the key in
    column key_col).  pack = (key_base, other_base).  Asynchronous."""
    lib = _lib.load()
    n = _packed_rows(packed, "packed")
    out = torch.empty((n, 2), dtype=torch.int64, device=packed.device) if out is None else \
        _out(out, "out", n, 2, packed)
    _lib.check(lib.smj_dev_unpack_rows(_ptr(packed), n, int(key_col), int(pack[0]), int(pack[1]), _ptr(out),
                                       _stream(stream)), "smj_dev_unpack_rows")
    return out


def _sort_merge_join_typed(lib, R, S, key1, key2, select1, select2, R_sorted, S_sorted, out, stream, key_type):
    for name, t in (("R", R), ("S", S)):
        if not (t.is_cuda and t.dim() == 2 and t.is_contiguous() and t.element_size() == 8):
            raise ValueError(f"{name}: contiguous 2-D 8-byte CUDA tensor required")
    nr, c1 = R.shape
    ns, c2 = S.shape
    R_sorted = torch.empty_like(R) if R_sorted is None else _out(R_sorted, "R_sorted", nr, c1, R, R.dtype)
    S_sorted = torch.empty_like(S) if S_sorted is None else _out(S_sorted, "S_sorted", ns, c2, R, S.dtype)
    if out is None:
        out = torch.empty((max(min(nr, ns), 1), c1 + c2 - 1), dtype=R.dtype, device=R.device)
    else:
        _out(out, "out", min(nr, ns), c1 + c2 - 1, R, R.dtype)
    rows = (ctypes.c_int64 * 3)()
    s1 = select1 or (0, 0)
    s2 = select2 or (0, 0)
    _lib.check(lib.smj_dev_sort_merge_join_typed(key_type, _ptr(R), nr, c1, int(select1 is not None), s1[0],
                                                 _bits(s1[1], key_type), key1, _ptr(S), ns, c2,
                                                 int(select2 is not None), s2[0], _bits(s2[1], key_type), key2,
                                                 _ptr(R_sorted), _ptr(S_sorted), _ptr(out), rows, _stream(stream)),
               "smj_dev_sort_merge_join_typed")
    return R_sorted[: rows[0]], S_sorted[: rows[1]], out[: rows[2]]


def msd_stats():
    """(single-key groups, LSD-fallback groups, m_R, m_S) of the last MSD pipeline call."""
    out = (ctypes.c_int64 * 4)()
    _lib.load().smj_debug_msd_stats(out)
    return tuple(int(v) for v in out)


def msd_packb():
    """1 if the last MSD pipeline call wrote packed pass-B rows (one 8-B word
    per row, MsdPlan::packB in smj_internal.h), else 0."""
    lib = _lib.load()
    lib.smj_debug_msd_packb.restype = ctypes.c_int64
    return int(lib.smj_debug_msd_packb())


def msd_wstage():
    """Groups of the last MSD pipeline call sorted by the wide-span staged
    kernel (msd_final_wstage_kernel: key spans over 4096 values)."""
    lib = _lib.load()
    if not hasattr(lib, "smj_debug_msd_wstage"):
        return 0
    lib.smj_debug_msd_wstage.restype = ctypes.c_int64
    return int(lib.smj_debug_msd_wstage())


def msd_segmented():
    """Pass-A buckets of the last MSD pipeline call given a segmented pass-B
    digit (MsdSeg in smj_internal.h: keys in dense intervals with wide gaps
    between, e.g. clustered keys)."""
    lib = _lib.load()
    if not hasattr(lib, "smj_debug_msd_segmented"):
        return 0
    lib.smj_debug_msd_segmented.restype = ctypes.c_int64
    return int(lib.smj_debug_msd_segmented())


def debug_wide_maxrun(rows=-1):
    """Diagnostic: the wide-span staged kernel hands a group to the radix tier
    when one of its bins holds more than `rows` rows (-1: the built-in limit;
    0: every group)."""
    _lib.load().smj_debug_wide_maxrun(int(rows))


def msd_bigdev():
    """Oversized multi-key groups of the last MSD pipeline call sorted on the
    device (msd_big_stage_kernel); the other oversized ones took the host-driven
    fallback."""
    lib = _lib.load()
    if not hasattr(lib, "smj_debug_msd_bigdev"):
        return 0
    lib.smj_debug_msd_bigdev.restype = ctypes.c_int64
    return int(lib.smj_debug_msd_bigdev())


def msd_groups():
    """(dense groups, radix-tier groups, wide-tier groups, in-LDS LSD groups) of the
    last MSD pipeline call."""
    out = (ctypes.c_int64 * 4)()
    lib = _lib.load()
    if hasattr(lib, "smj_debug_msd_tiers"):
        lib.smj_debug_msd_tiers(out)
    else:  # an older build under SMJ_LIB (A/B): no in-LDS LSD count
        lib.smj_debug_msd_groups(out)
    return tuple(int(v) for v in out)


def force_parts(parts=0):
    """Diagnostic: run every pipeline call in the partitioned mode with `parts`
    key-range parts (0 = automatic: only tables over 1.6e8 rows are split, kMsdSingleMax)."""
    _lib.load().smj_debug_force_parts(int(parts))


def biased_base(key_base):
    return int(key_base) & ((1 << 64) - 1)


def select(table, select_col, select_val, out=None, stream=None):
    """Stable compaction: rows with table[:, select_col] > select_val."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    out = torch.empty_like(table) if out is None else _out(out, "out", n, cols, table)
    m = ctypes.c_int64(0)
    _lib.check(lib.smj_dev_select(_ptr(table), n, cols, select_col, int(select_val), _ptr(out),
                                  ctypes.byref(m), _stream(stream)), "smj_dev_select")
    return out[: m.value]


def merge(a, b, key_col=0, out=None, stream=None):
    """Stable merge of two runs sorted on key_col (a's rows first on ties)."""
    lib = _lib.load()
    _table(a, "a")
    _table(b, "b")
    if a.shape[1] != b.shape[1]:
        raise ValueError("runs must have the same column count")
    if out is None:
        out = torch.empty((a.shape[0] + b.shape[0], a.shape[1]), dtype=torch.int64, device=a.device)
    else:
        _out(out, "out", a.shape[0] + b.shape[0], a.shape[1], a)
    _lib.check(lib.smj_dev_merge(_ptr(a), a.shape[0], _ptr(b), b.shape[0], a.shape[1], key_col, _ptr(out),
                                 _stream(stream)), "smj_dev_merge")
    return out


def join(R, S, key1=0, key2=0, out=None, count=None, sync=True, stream=None):
    """1:1 zip merge join of sorted R and S.  Returns out[:J] when sync, else
    (out, count) with the row count left on the device in `count`."""
    lib = _lib.load()
    _table(R, "R")
    _table(S, "S")
    nr, c1 = R.shape
    ns, c2 = S.shape
    tc = c1 + c2 - 1
    if out is None:
        out = torch.empty((max(min(nr, ns), 1), tc), dtype=torch.int64, device=R.device)
    else:
        _out(out, "out", min(nr, ns), tc, R)
    if count is None:
        count = torch.zeros(1, dtype=torch.int64, device=R.device)
    j = ctypes.c_int64(0)
    _lib.check(lib.smj_dev_join(_ptr(R), nr, c1, _ptr(S), ns, c2, key1, key2, _ptr(out),
                                ctypes.c_void_p(count.data_ptr()), ctypes.byref(j) if sync else None,
                                _stream(stream)), "smj_dev_join")
    if sync:
        return out[: j.value]
    return out, count


def partition_count(table, splitters, key_col=0, select_col=0, select_val=None, stream=None):
    """Rows per destination bucket (bucket(k) = #{splitters < k}) + (min, max)
    of the selected keys.  splitters: 1-D int64 CUDA tensor, sorted."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    ns = int(splitters.numel())
    counts = (ctypes.c_int64 * (ns + 1))()
    mm = (ctypes.c_int64 * 2)()
    use = select_val is not None
    _lib.check(lib.smj_dev_partition_count(_ptr(table), n, cols, int(use), select_col,
                                           int(select_val) if use else 0, key_col, _ptr(splitters), ns,
                                           counts, mm, _stream(stream)), "smj_dev_partition_count")
    return [int(c) for c in counts], (int(mm[0]), int(mm[1]))


def partition_scatter(table, splitters, counts, key_col=0, select_col=0, select_val=None, out=None,
                      stream=None):
    """Stable scatter of the selected rows into bucket-contiguous order."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    total = sum(counts)
    if out is None:
        out = torch.empty((max(total, 1), cols), dtype=torch.int64, device=table.device)
    else:
        _out(out, "out", total, cols, table)
    c = (ctypes.c_int64 * len(counts))(*counts)
    use = select_val is not None
    _lib.check(lib.smj_dev_partition_scatter(_ptr(table), n, cols, int(use), select_col,
                                             int(select_val) if use else 0, key_col, _ptr(splitters),
                                             int(splitters.numel()), c, _ptr(out), _stream(stream)),
               "smj_dev_partition_scatter")
    return out[:total]


def partition(table, splitters, key_col=0, select_col=0, select_val=None, out=None, stream=None):
    """Stable select + bucket scatter in one call (smj_dev_partition): returns
    (bucket counts, the selected rows in bucket-contiguous order)."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    ns = int(splitters.numel())
    if out is None:
        out = torch.empty((max(n, 1), cols), dtype=torch.int64, device=table.device)
    else:
        _out(out, "out", n, cols, table)
    counts = (ctypes.c_int64 * (ns + 1))()
    use = select_val is not None
    _lib.check(lib.smj_dev_partition(_ptr(table), n, cols, int(use), select_col, int(select_val) if use else 0,
                                     key_col, _ptr(splitters), ns, _ptr(out), counts, _stream(stream)),
               "smj_dev_partition")
    counts = [int(c) for c in counts]
    return counts, out[: sum(counts)]


def _host_splitters(bounds):
    arr = (ctypes.c_int64 * max(len(bounds), 1))(*[int(b) for b in bounds])
    return arr, len(bounds)


def partition_plan(table, bounds, counts, key_col=0, select_col=0, select_val=None, stream=None):
    """Asynchronous first half of the partition (smj_dev_partition_plan):
    per-(chunk, bucket) counts of the selected rows turned into stable output
    starts; the len(bounds) + 1 bucket counts are written into `counts` (a
    1-D int64 CUDA tensor view) without a host synchronisation.  bounds: a
    sorted host list.  Returns the plan (a device buffer) for
    partition_apply."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    if not (counts.is_cuda and counts.dtype == torch.int64 and counts.is_contiguous()
            and counts.numel() == len(bounds) + 1):
        raise ValueError("counts must be a contiguous int64 CUDA tensor of len(bounds) + 1 entries")
    plan = torch.empty(max(int(lib.smj_partition_plan_bytes(n, cols, len(bounds))), 4) // 4, dtype=torch.int32,
                       device=table.device)
    spl, ns = _host_splitters(bounds)
    use = select_val is not None
    _lib.check(lib.smj_dev_partition_plan(_ptr(table), n, cols, int(use), select_col, int(select_val) if use else 0,
                                          key_col, spl, ns, _ptr(plan), ctypes.c_void_p(counts.data_ptr()),
                                          _stream(stream)), "smj_dev_partition_plan")
    return plan


def partition_apply(table, bounds, plan, key_col=0, select_col=0, select_val=None, out=None, stream=None):
    """Asynchronous second half: the selected rows in bucket-contiguous order,
    written into `out` (n rows of room; the caller knows the selected count
    from the plan's counts).  Returns out."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    out = torch.empty((max(n, 1), cols), dtype=torch.int64, device=table.device) if out is None else \
        _out(out, "out", n, cols, table)
    spl, ns = _host_splitters(bounds)
    use = select_val is not None
    _lib.check(lib.smj_dev_partition_apply(_ptr(table), n, cols, int(use), select_col,
                                           int(select_val) if use else 0, key_col, spl, ns, _ptr(plan), _ptr(out),
                                           _stream(stream)), "smj_dev_partition_apply")
    return out


def region_capacities(sample_keys, n, bounds, tile=4096, sigmas=8.0):
    """Region starts / capacities (rows) for partition_regions from a key
    sample of the table (host list): bucket b's estimated rows + sigmas binomial
    standard deviations + one tile, capped at n (as msd_part1 sizes the
    partitioned mode's regions).  Returns (h_region list of 2 (nb) ints, rows
    the output buffer needs)."""
    import numpy as np
    nb = len(bounds) + 1
    sample_keys = np.asarray(sample_keys, dtype=np.int64)
    m = len(sample_keys)
    if m == 0:
        caps = np.full(nb, n, dtype=np.int64)
    else:  # (vectorised: this runs between the splitters' host copy and the first partition launch)
        f = np.bincount(np.searchsorted(np.asarray(bounds, dtype=np.int64), sample_keys, side="left"),
                        minlength=nb) / m
        sd = n / m * np.sqrt(m * f * (1.0 - f) + 1.0)
        caps = np.minimum(n, (n * f + sigmas * sd).astype(np.int64) + tile)
    ends = np.cumsum(caps)
    return (ends - caps).tolist() + caps.tolist(), int(ends[-1])


def partition_regions(table, bounds, region, counts, key_col=0, select_col=0, select_val=None, out=None,
                      stream=None, pack=None):
    """One-read stable partition (smj_dev_partition_regions): bucket b's rows
    at out[region[b]: region[b] + count_b]; `counts` (a 1-D int64 CUDA tensor of
    len(bounds) + 2 entries) gets the exact counts and, last, the overflow /
    timeout flag word.  pack = (key_base, other_base) for a 2-column table:
    out holds one packed word per row (smj_dev_partition_regions_pk; flag bit
    2 = a row did not fit, out unusable).  Asynchronous.  Returns out."""
    lib = _lib.load()
    _table(table, "table")
    n, cols = table.shape
    nb = len(bounds) + 1
    if len(region) != 2 * nb:
        raise ValueError("region must hold 2 (len(bounds) + 1) entries")
    need = max(region[b] + region[nb + b] for b in range(nb)) if n else 0
    if not (counts.is_cuda and counts.dtype == torch.int64 and counts.is_contiguous() and counts.numel() == nb + 1):
        raise ValueError("counts must be a contiguous int64 CUDA tensor of len(bounds) + 2 entries")
    if pack is not None and cols != 2:
        raise ValueError("packed partitions take 2-column tables")
    oc = 1 if pack is not None else cols
    out = torch.empty((max(need, 1), oc), dtype=torch.int64, device=table.device) if out is None else \
        _out(out, "out", need, oc, table)
    spl, ns = _host_splitters(bounds)
    reg = (ctypes.c_int64 * len(region))(*[int(v) for v in region])
    use = select_val is not None
    if pack is not None:
        _lib.check(lib.smj_dev_partition_regions_pk(_ptr(table), n, int(use), select_col, int(select_val) if use else 0,
                                                    key_col, spl, ns, reg, _ptr(out), ctypes.c_void_p(counts.data_ptr()),
                                                    int(pack[0]), int(pack[1]), _stream(stream)),
                   "smj_dev_partition_regions_pk")
        return out
    _lib.check(lib.smj_dev_partition_regions(_ptr(table), n, cols, int(use), select_col,
                                             int(select_val) if use else 0, key_col, spl, ns, reg, _ptr(out),
                                             ctypes.c_void_p(counts.data_ptr()), _stream(stream)),
               "smj_dev_partition_regions")
    return out


def gen_uniform(rows, row0=0, seed=1, key_range=None, device="cuda", out=None, stream=None):
    """Synthetic (key, payload) table: keys iid uniform in [1, key_range],
    payload = global row index."""
    lib = _lib.load()
    if key_range is None:
        key_range = 3 * rows
    if out is None:
        out = torch.empty((rows, 2), dtype=torch.int64, device=device)
    _lib.check(lib.smj_dev_gen_uniform(_ptr(out), row0, rows, seed, key_range, _stream(stream)),
               "smj_dev_gen_uniform")
    return out


def gen_zipf(rows, row0=0, seed=3, domain=100_000_000, theta=0.9, device="cuda", out=None, stream=None):
    """Synthetic Zipf(theta) keys over [1, domain]."""
    lib = _lib.load()
    zeta = lib.smj_zipf_zeta(domain, theta)
    if out is None:
        out = torch.empty((rows, 2), dtype=torch.int64, device=device)
    _lib.check(lib.smj_dev_gen_zipf(_ptr(out), row0, rows, seed, domain, theta, zeta, _stream(stream)),
               "smj_dev_gen_zipf")
    return out


def gen_wide(rows, row0=0, seed=1, plant_seed=1, plant_rows=0, device="cuda", out=None, stream=None):
    """C3-wide synthetic table (SURVEY 8(d) stress input): full-range signed
    int64 keys; with plant_rows > 0 a random third of the rows take the key of
    a random row of the plant_seed table of plant_rows rows (R), so they join.
    payload = global row index (smj_dev_gen_wide)."""
    lib = _lib.load()
    if out is None:
        out = torch.empty((rows, 2), dtype=torch.int64, device=device)
    _lib.check(lib.smj_dev_gen_wide(_ptr(out), int(row0), int(rows), int(seed), int(plant_seed), int(plant_rows),
                                    _stream(stream)), "smj_dev_gen_wide")
    return out


MASK64 = (1 << 64) - 1


DIST_HDR = 5  # smj.h smj_dev_dist_sample: [valid samples, samples of R, of S, rows of R, of S]


def dist_sample(R, S, key_R, key_S, samples, out=None, stream=None):
    """smj_dev_dist_sample: this rank's splitter sample of R and S (evenly
    spaced rows, R's then S's keys after a 5-word header, INT64_MAX pads) in
    a device int64 vector of 5 + 2 samples words.  Asynchronous."""
    lib = _lib.load()
    _table(R, "R")
    _table(S, "S")
    n = DIST_HDR + 2 * samples
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=R.device)
    elif not (out.is_cuda and out.dtype == torch.int64 and out.is_contiguous() and out.numel() >= n):
        raise ValueError(f"out must be a contiguous int64 CUDA tensor of >= {n} entries")
    _lib.check(lib.smj_dev_dist_sample(_ptr(R), R.shape[0], R.shape[1], key_R, _ptr(S), S.shape[0], S.shape[1],
                                       key_S, int(samples), ctypes.c_void_p(out.data_ptr()), _stream(stream)),
               "smj_dev_dist_sample")
    return out


def dist_splitters(gathered, world, stride, parts, q20=None, out=None, stream=None):
    """smj_dev_dist_splitters: from the world gathered sample buffers
    (`gathered`, world * stride int64 words on the device), the parts - 1
    splitters then L (the ranks' valid samples) into `out` (parts int64 words,
    device).  q20: the cumulative stage fractions << 20 (host ints) or None
    for equal parts.  Asynchronous."""
    lib = _lib.load()
    if not (gathered.is_cuda and gathered.dtype == torch.int64 and gathered.is_contiguous()
            and gathered.numel() >= world * stride):
        raise ValueError("gathered must be a contiguous int64 CUDA tensor of world * stride entries")
    if out is None:
        out = torch.empty(parts, dtype=torch.int64, device=gathered.device)
    elif not (out.is_cuda and out.dtype == torch.int64 and out.is_contiguous() and out.numel() >= parts):
        raise ValueError(f"out must be a contiguous int64 CUDA tensor of >= {parts} entries")
    q = None
    if q20 is not None:
        if len(q20) != parts - 1:
            raise ValueError("q20 needs parts - 1 entries")
        q = (ctypes.c_int * max(1, len(q20)))(*[int(v) for v in q20])
    _lib.check(lib.smj_dev_dist_splitters(ctypes.c_void_p(gathered.data_ptr()), int(world), int(stride), int(parts), q,
                                          ctypes.c_void_p(out.data_ptr()), _stream(stream)),
               "smj_dev_dist_splitters")
    return out


def digest_async(table, pos0=0, out=None, stream=None):
    """smj_dev_digest of `table` (rows at global positions pos0, pos0 + 1, ...)
    into out (a 1-element int64 CUDA tensor holding the uint64 bits;
    allocated if None), without a host synchronisation.  Returns out."""
    lib = _lib.load()
    if not (isinstance(table, torch.Tensor) and table.is_cuda and table.element_size() == 8 and table.dim() == 2
            and table.is_contiguous()):
        raise ValueError("table must be a contiguous 2-D 8-byte CUDA tensor")
    if out is None:
        out = torch.empty(1, dtype=torch.int64, device=table.device)
    _lib.check(lib.smj_dev_digest(_ptr(table), table.shape[0], max(table.shape[1], 1), int(pos0),
                                  ctypes.c_void_p(out.data_ptr()), _stream(stream)), "smj_dev_digest")
    return out


def digest(table, pos0=0, stream=None):
    """The order-sensitive digest of `table` as a Python int in [0, 2^64):
    digests of consecutive slices at their global positions add up (mod 2^64)
    to the digest of the whole table (smj.h smj_dev_digest)."""
    d = digest_async(table, pos0, stream=stream)
    return int(d.item()) & MASK64


def trim():
    """smj_trim: return every device buffer the library holds (synchronises)."""
    _lib.check(_lib.load().smj_trim(), "smj_trim")


def scratch_bytes():
    """Device bytes the library holds now (smj_scratch_bytes)."""
    return int(_lib.load().smj_scratch_bytes())


def set_scratch_limit(nbytes=-1):
    """smj_set_scratch_limit: a call ending over `nbytes` of library scratch
    trims before it returns (-1: keep scratch for the next call)."""
    _lib.load().smj_set_scratch_limit(int(nbytes))


def prof_enable(on=True):
    _lib.load().smj_prof_enable(int(bool(on)))


def prof_report():
    """{kernel: {"launches", "ms", "bytes"}} since the last report."""
    lib = _lib.load()
    need = lib.smj_prof_report(None, 0)
    buf = ctypes.create_string_buffer(max(need, 2))
    lib.smj_prof_report(buf, len(buf))
    return json.loads(buf.value.decode())
