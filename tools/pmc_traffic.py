#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC runs (FETCH_SIZE and WRITE_SIZE
collected in SEPARATE passes, MI355X_MICROARCH.md "rocprofv3 PMC slots").

    python tools/pmc_traffic.py gpurun_out/r01b/pmc_fetch gpurun_out/r01b/pmc_write \
        --rows 100000000 -o profiles/pmc_traffic.json

gfx950 corrections (MI355X_MICROARCH.md section HBM): FETCH_SIZE reports half
the bytes of a wide coalesced stream, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane stores.  Both counters are in KiB per dispatch.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

TAGS = [  # (regex on the demangled kernel name, profiler tag used by bench.py)
    (r"chunk_scatter_kernel<\d+, 10,", "radix_scatter"),
    (r"chunk_hist_kernel<\d+, 10,", "radix_hist"),
    (r"chunk_scatter_kernel<\d+, 0,", "select_scatter"),
    (r"chunk_hist_kernel<\d+, 0,", "select_hist"),
    (r"chunk_scatter_kernel<\d+, 4,", "partition_scatter"),
    (r"chunk_hist_kernel<\d+, 4,", "partition_hist"),
    (r"chunk_scan_(seg|apply)_kernel", "radix_scan"),
    (r"hist_radix_kernel", "hist_radix"),
    (r"join_tile_kernel", "join_tiles"),
    (r"join_compact_kernel", "join_compact"),
    (r"join_scan_kernel", "join_scan"),
    (r"merge_partition_kernel", "join_partition"),
    (r"merge_tile_kernel", "merge_tiles"),
    (r"gen_uniform_kernel", "gen_uniform"),
    (r"plan_kernel", "plan"),
]


def tag_of(name):
    for rx, tag in TAGS:
        if re.search(rx, name):
            return tag
    return None


def read_counter(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                t = tag_of(row.get("Kernel_Name", ""))
                if t:
                    per[t].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("-o", "--out", default="profiles/pmc_traffic.json")
    a = ap.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for t in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(t, [0])) / max(len(fetch.get(t, [])), 1)
        w = sum(write.get(t, [0])) / max(len(write.get(t, [])), 1)
        kernels[t] = {"dispatches": len(fetch.get(t, [])), "fetch_kib_raw": round(f, 1),
                      "write_kib": round(w, 1), "hbm_bytes_per_launch": round((2 * f + w) * 1024)}
    out = {"rows_per_table": a.rows, "source": [a.fetch_dir, a.write_dir],
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB per dispatch (gfx950: FETCH_SIZE "
                         "counts half of a wide coalesced read; MI355X_MICROARCH.md, HBM)",
           "kernels": kernels}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for t, k in kernels.items():
        print(f"{t:20s} {k['hbm_bytes_per_launch'] / 1e9:8.3f} GB/launch  ({k['dispatches']} dispatches)")


if __name__ == "__main__":
    main()
