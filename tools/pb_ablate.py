"""part_b ablation on the C3 workload: re-runs the last pipeline call's part_b
launches with ablation bits (smj_msd.hip) and prints ms per round (R + S).

    python tools/pb_ablate.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch  # noqa: E402

from smj import _lib, ops  # noqa: E402

lib = _lib.load()
lib.smj_debug_part_b_time.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
n = int(float(os.environ.get("ROWS", "1e8")))
R = ops.gen_uniform(n, seed=1, key_range=3 * n)
S = ops.gen_uniform(n, seed=2, key_range=3 * n)
ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000))
torch.cuda.synchronize()
ms = ctypes.c_float()
variants = [(0, "baseline"), (64, "1 workgroup per CU"), (66, "1 WG/CU, no row stores"), (2, "no row stores"), (8, "no offs stores"), (10, "no stores at all"),
            (4, "synthetic rows (no gathers)"), (6, "no gathers, no row stores"), (14, "no global traffic"),
            (16, "ballot ranking path (forced)"), (30, "no traffic, ballot path"), (46, "no traffic, no lookups")]
for dbg, name in variants:
    assert lib.smj_debug_part_b_time(dbg, 10, ctypes.byref(ms)) == 0
    print(f"dbg {dbg:2d} {name:30s} {ms.value:.3f} ms (R + S)", flush=True)
