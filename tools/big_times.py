"""Where msd_big_stage_kernel's time goes on C5 (oversized Zipf groups): per
size class (log2 of the larger table's rows) the groups and the workgroup
cycles they took, and the cycles per phase.  Needs the SMJ_STAMPS build:

    tools/build_variant.sh stamps -DSMJ_STAMPS=1
    SMJ_LIB=pim-sort-merge-join_amd/lib/variants/stamps/libsmj_hip.so SMJ_DEBUG_BIG=1 python tools/big_times.py
"""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))

import torch  # noqa: E402

from smj import _lib, ops  # noqa: E402


def main():
    nr, ns = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000, int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
    R = ops.gen_zipf(nr, seed=3, domain=100_000_000, theta=0.9)
    S = ops.gen_zipf(ns, seed=4, domain=100_000_000, theta=0.9)
    bufs = dict(R_sorted=torch.empty_like(R), S_sorted=torch.empty_like(S),
                out=torch.empty((nr, 3), dtype=torch.int64, device=R.device))
    lib = _lib.load()
    out = (ctypes.c_ulonglong * 72)()
    ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), **bufs)
    torch.cuda.synchronize()
    lib.smj_debug_big_times(out)  # reset
    ops.prof_enable(True)
    ops.prof_report()
    t0 = time.perf_counter()
    ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000), **bufs)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    prof = ops.prof_report()
    lib.smj_debug_big_times(out)
    cyc = list(out[:32])
    cnt = list(out[32:64])
    ph = list(out[64:69])
    tot = sum(cyc) or 1
    res = {"wall_ms": round(wall, 2), "msd_big_dev_ms": round(prof.get("msd_big_dev", {}).get("ms", 0), 3),
           "classes": {f"2^{c}": {"groups": cnt[c], "cycles": cyc[c], "share": round(cyc[c] / tot, 4),
                                  "cycles_per_group": round(cyc[c] / max(cnt[c], 1))}
                       for c in range(32) if cnt[c]},
           "phases": dict(zip(["lists", "count", "starts", "scatter", "join"],
                              [round(v / max(sum(ph), 1), 4) for v in ph]))}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
