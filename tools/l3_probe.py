"""Per-row cost of the MSD passes against table size: does a pass whose input
is still resident in the 256 MiB Infinity Cache (small tables, re-run
back-to-back) run faster per row than at C3 size?  Re-runs the last pipeline
call's part_b / final launches (smj_debug_part_b_time / smj_debug_final_time).

    python tools/l3_probe.py
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pim-sort-merge-join_amd"))
import torch  # noqa: E402

from smj import _lib, ops  # noqa: E402

lib = _lib.load()
for f in ("smj_debug_final_time", "smj_debug_part_b_time"):
    getattr(lib, f).argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
sizes = [int(float(x)) for x in os.environ.get("SIZES", "1e6,2e6,4e6,8e6,16e6,32e6,1e8").split(",")]
for n in sizes:
    R = ops.gen_uniform(n, seed=1, key_range=3 * n)
    S = ops.gen_uniform(n, seed=2, key_range=3 * n)
    bufs = (torch.empty_like(R), torch.empty_like(S), torch.empty((n, 3), dtype=torch.int64, device=R.device))
    for _ in range(2):
        ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), *bufs)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), *bufs)
    b.record()
    torch.cuda.synchronize()
    full = a.elapsed_time(b) / 5
    fin, pb = ctypes.c_float(), ctypes.c_float()
    assert lib.smj_debug_final_time(0, 10, ctypes.byref(fin)) == 0
    assert lib.smj_debug_part_b_time(0, 10, ctypes.byref(pb)) == 0
    rows = 2 * n
    print(f"n={n:>11,d}  step {full:8.3f} ms ({full * 1e6 / rows:6.3f} ns/row)  "
          f"final {fin.value:7.3f} ms ({fin.value * 1e6 / rows:6.3f} ns/row)  "
          f"part_b {pb.value:7.3f} ms ({pb.value * 1e6 / rows:6.3f} ns/row)  groups {ops.msd_groups()}", flush=True)
    del R, S, bufs
    torch.cuda.empty_cache()
