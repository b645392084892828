"""smj -- MI355X sort-merge-join (Python host side of libsmj_hip.so).

Layout of the package directory `pim-sort-merge-join_amd/`:
  csrc/   HIP kernels (gfx950) + the C-ABI (include/smj.h)
  host/   the C host program smj_app (drop-in for the reference app.c) + CSV I/O
  smj/    this package: ctypes binding, torch-level ops, the multi-GPU driver
"""
from ._lib import LIB_PATH, APP_PATH, SmjError, build, load  # noqa: F401

__all__ = ["LIB_PATH", "APP_PATH", "SmjError", "build", "load"]
