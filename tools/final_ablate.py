"""Staged final kernel ablation on the C3 workload: re-runs the last pipeline
call's final launches with ablation bits (smj_msd.hip launch_msd_final).

    python tools/final_ablate.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch  # noqa: E402

from smj import _lib, ops  # noqa: E402

lib = _lib.load()
lib.smj_debug_final_time.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
n = int(float(os.environ.get("ROWS", "1e8")))
R = ops.gen_uniform(n, seed=1, key_range=3 * n)
S = ops.gen_uniform(n, seed=2, key_range=3 * n)
ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000))
torch.cuda.synchronize()
ms = ctypes.c_float()
CASES = [(0, "baseline"), (64, "1 workgroup per CU"), (2, "no sorted-row stores"), (8, "no join rows"),
         (10, "no stores at all"), (4, "synthetic rows (no gathers)"), (14, "no gathers, no stores"),
         (16, "no equal-key rounds"), (30, "no gathers/stores/rounds"), (0, "baseline")]
if os.environ.get("DBG"):  # e.g. DBG=0,2,8
    CASES = [(int(b), f"bits {b}") for b in os.environ["DBG"].split(",")]
for dbg, name in CASES:
    assert lib.smj_debug_final_time(dbg, 5, ctypes.byref(ms)) == 0
    print(f"dbg {dbg:2d} {name:28s} {ms.value:.3f} ms", flush=True)
