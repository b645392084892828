"""ctypes binding of libsmj_hip.so (the C-ABI declared in include/smj.h).

This is the Python-side twin of the cgo/JNI-style stubs in INTEGRATION.md:
plain pointers and sizes, no torch types cross the boundary.  The library is
the product path -- there is no fallback: if it is missing or fails to load,
every call raises.
"""
import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("SMJ_LIB") or os.path.join(PKG_DIR, "lib", "libsmj_hip.so")
CSV_LIB_PATH = os.path.join(PKG_DIR, "lib", "libsmj_csv.so")
APP_PATH = os.path.join(PKG_DIR, "bin", "smj_app")

SMJ_OK = 0
ERRORS = {
    -1: "SMJ_ERR_INVALID", -2: "SMJ_ERR_HIP", -3: "SMJ_ERR_NOMEM", -4: "SMJ_ERR_NODEVICE",
    -5: "SMJ_ERR_TOO_LARGE", -6: "SMJ_ERR_TIMEOUT", -7: "SMJ_ERR_UNSUPPORTED",
}

# exported symbol -> (restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_U = ctypes.c_uint64
_D = ctypes.c_double
_PL = ctypes.POINTER(ctypes.c_int64)
_PI = ctypes.POINTER(ctypes.c_int)

SIGNATURES = {
    "smj_strerror": (ctypes.c_char_p, [_I]),
    "smj_version": (ctypes.c_char_p, []),
    "smj_init": (_I, [_I]),
    "smj_init_devices": (_I, [_PI, _I]),
    "smj_device_count": (_I, []),
    "smj_finalize": (None, []),
    "smj_select": (_I, [_P, _P, _P, _I, _L, _PI]),
    "smj_sort": (_I, [_P, _P, _I]),
    "smj_merge": (_I, [_P, _P, _P, _P, _I, _P]),
    "smj_join": (_I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(_P), _PL]),
    "smj_sort_merge_join": (_I, [_P, _P, _P, _P, _I, _L, _I, _L, _I, _I, ctypes.POINTER(_P), _PL, _P]),
    "smj_dev_select_sort": (_I, [_P, _L, _I, _I, _I, _L, _I, _U, _P, _PL, _P]),
    "smj_dev_select_sort_lsd": (_I, [_P, _L, _I, _I, _I, _L, _I, _U, _P, _PL, _P]),
    "smj_dev_sort_merge_join": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _L, _I, _I, _I, _L, _I, _P, _P, _P, _PL, _P]),
    "smj_dev_sort_merge_join_begin": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _L, _I, _I, _I, _L, _I, _P, _P, _P,
                                           ctypes.POINTER(ctypes.c_void_p)]),
    "smj_dev_sort_merge_join_end": (_I, [_P, _P, _PL]),
    "smj_dev_sort_merge_join_typed": (_I, [_I, _P, _L, _I, _I, _I, ctypes.c_uint64, _I, _P, _L, _I, _I, _I,
                                           ctypes.c_uint64, _I, _P, _P, _P, _PL, _P]),
    "smj_sort_merge_join_typed": (_I, [_I, _P, _P, _P, _P, _I, ctypes.c_uint64, _I, ctypes.c_uint64, _I, _I,
                                       ctypes.POINTER(_P), _PL, _P]),
    "smj_dev_select": (_I, [_P, _L, _I, _I, _L, _P, _PL, _P]),
    "smj_dev_merge": (_I, [_P, _L, _P, _L, _I, _I, _P, _P]),
    "smj_dev_join": (_I, [_P, _L, _I, _P, _L, _I, _I, _I, _P, _P, _PL, _P]),
    "smj_dev_partition_count": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _I, _PL, _PL, _P]),
    "smj_dev_partition_scatter": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _I, _PL, _P, _P]),
    "smj_dev_partition": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _I, _P, _PL, _P]),
    "smj_partition_plan_bytes": (ctypes.c_size_t, [_L, _I, _I]),
    "smj_dev_partition_plan": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _I, _P, _P, _P]),
    "smj_dev_partition_apply": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _I, _P, _P, _P]),
    "smj_dev_partition_regions": (_I, [_P, _L, _I, _I, _I, _L, _I, _P, _I, _P, _P, _P, _P]),
    "smj_dev_gen_uniform": (_I, [_P, _L, _L, _U, _U, _P]),
    "smj_dev_gen_zipf": (_I, [_P, _L, _L, _U, _L, _D, _D, _P]),
    "smj_dev_gen_wide": (_I, [_P, _L, _L, _U, _U, _L, _P]),
    "smj_trim": (_I, []),
    "smj_scratch_bytes": (_L, []),
    "smj_set_scratch_limit": (None, [_L]),
    "smj_zipf_zeta": (_D, [_L, _D]),
    "smj_dev_digest": (_I, [_P, _L, _I, _L, _P, _P]),
    "smj_dev_dist_sample": (_I, [_P, _L, _I, _I, _P, _L, _I, _I, _I, _P, _P]),
    "smj_dev_dist_splitters": (_I, [_P, _I, _L, _I, _PI, _P, _P]),
    "smj_dev_partition_regions_pk": (_I, [_P, _L, _I, _I, _L, _I, _P, _I, _P, _P, _P, _L, _L, _P]),
    "smj_dev_unpack_rows": (_I, [_P, _L, _I, _L, _L, _P, _P]),
    "smj_dev_sort_merge_join_begin_pk": (_I, [_P, _L, _I, _I, _L, _L, _P, _L, _I, _I, _L, _L, _P, _P, _P,
                                              ctypes.POINTER(ctypes.c_void_p)]),
    "smj_debug_msd_stats": (None, [_PL]),
    "smj_debug_msd_groups": (None, [_PL]),
    "smj_debug_msd_tiers": (None, [_PL]),
    "smj_debug_force_parts": (None, [_I]),
    "smj_debug_spin_limit": (None, [_L]),
    "smj_debug_shard_rows": (_I, [_PL, _I]),
    "smj_prof_enable": (None, [_I]),
    "smj_prof_report": (_I, [ctypes.c_char_p, ctypes.c_size_t]),
}


class SmjError(RuntimeError):
    def __init__(self, code, where):
        self.code = code
        super().__init__(f"{where}: {ERRORS.get(code, code)} ({code})")


_lock = threading.Lock()
_lib = None


def build(quiet=True):
    """Compile libsmj_hip.so / smj_app for gfx950 in-tree (hipcc cross-compiles)."""
    kw = dict(check=True, cwd=PKG_DIR)
    if quiet:
        kw.update(stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-j8"], **kw)


def load(build_if_missing=True):
    """Load libsmj_hip.so.  torch is imported first so that this library and
    torch share one HIP runtime (both need libamdhip64.so.7)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (HIP runtime first)
        if not os.path.exists(LIB_PATH) and build_if_missing:
            build()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `make -C {PKG_DIR}`")
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("SMJ_LIB") and not hasattr(lib, name):
                continue  # an older build loaded for a same-box A/B (tools/ab.sh)
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def source_sha():
    """sha256 (16 hex digits) of the library's sources (csrc/, include/): the
    key under which a profile summary (profiles/pmc_traffic*.json) is valid
    for the library built from this tree."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*")) + glob.glob(os.path.join(REPO_DIR, "include", "*.h")))
    for f in files:
        h.update(os.path.relpath(f, REPO_DIR).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check(rc, where):
    if rc != SMJ_OK:
        raise SmjError(rc, where)
    return rc
