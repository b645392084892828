"""Host-pointer path timing buckets (app.c:763-772: CPU-GPU / GPU / GPU-CPU)
with the staged input (chunked H2D copies overlapping part_a, the default)
against one copy per table (SMJ_STAGED=0), on the bundled CSVs' sizes, C2
(1M x 1M) and C3-sized host tables (1e8 x 1e8).

    python tools/h2d_overlap.py            (runs both modes as subprocesses)
"""
import ctypes
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))


class Block(ctypes.Structure):
    _fields_ = [("table_num", ctypes.c_int), ("col_num", ctypes.c_int), ("row_num", ctypes.c_int)]


class Timing(ctypes.Structure):
    _fields_ = [("cpu_gpu_ms", ctypes.c_double), ("gpu_ms", ctypes.c_double), ("gpu_cpu_ms", ctypes.c_double)]


def child():
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime)
    from smj import _lib
    lib = _lib.load()
    assert lib.smj_init(1) == 1
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    out = []
    for name, n in (("bundled-size 1e5", 100_000), ("C2 1e6", 1_000_000), ("C3 1e8", 100_000_000)):
        rng = np.random.default_rng(1)
        R = np.empty((n, 2), dtype=np.int64)
        S = np.empty((n, 2), dtype=np.int64)
        R[:, 0] = rng.integers(1, 3 * n, n)
        S[:, 0] = rng.integers(1, 3 * n, n)
        R[:, 1] = np.arange(n)
        S[:, 1] = np.arange(n)
        bR, bS = Block(0, 2, n), Block(1, 2, n)
        best = None
        for rep in range(4):
            res, rows, tm = ctypes.c_void_p(), ctypes.c_int64(0), Timing()
            t0 = time.perf_counter()
            _lib.check(lib.smj_sort_merge_join(ctypes.byref(bR), R.ctypes.data_as(ctypes.c_void_p), ctypes.byref(bS),
                                               S.ctypes.data_as(ctypes.c_void_p), 0, 5000, 0, 5000, 0, 0,
                                               ctypes.byref(res), ctypes.byref(rows), ctypes.byref(tm)), "smj")
            wall = (time.perf_counter() - t0) * 1e3
            libc.free(res)
            rec = {"tables": name, "rows": n, "joined": rows.value, "cpu_gpu_ms": round(tm.cpu_gpu_ms, 3),
                   "gpu_ms": round(tm.gpu_ms, 3), "gpu_cpu_ms": round(tm.gpu_cpu_ms, 3), "wall_ms": round(wall, 3)}
            if rep > 0 and (best is None or wall < best["wall_ms"]):
                best = rec
        out.append(best)
    print(json.dumps(out))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        return child()
    result = {}
    for mode in ("1", "0"):
        env = dict(os.environ, SMJ_STAGED=mode)
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, check=True)
        result["staged" if mode == "1" else "serial"] = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(result, indent=1))


if __name__ == "__main__":
    main()
