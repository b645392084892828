#!/usr/bin/env python3
"""Per-profiler-scope HBM traffic from rocprofv3 PMC runs (FETCH_SIZE and
WRITE_SIZE collected in SEPARATE passes, MI355X_MICROARCH.md "rocprofv3 PMC
slots").

    python tools/pmc_traffic.py gpurun_out/r01g/pmc_fetch gpurun_out/r01g/pmc_write \
        --rows 100000000 -o profiles/pmc_traffic.json

bench.py times each pipeline stage with one HIP-event scope (smj_api.hip
ProfScope); a scope may launch several kernels (msd_final = staged LDS kernel
+ radix-list kernel + wide-key kernel).  Traffic per scope launch = the sum of
all its kernels' bytes / the dispatch count of the scope's PRIMARY kernel
(launched exactly once per scope).

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

TAGS = [  # (regex on the demangled kernel name, bench.py scope tag, primary?)
    (r"msd_final_stage_kernel", "msd_final", True),
    (r"msd_final_wstage64_kernel", "msd_final_tiers", True),   # (round 6: launched by msd_back when needed)
    (r"msd_final_wstage_kernel", "msd_final_tiers", False),
    (r"msd_final_kernel<2, 2>", "msd_final_tiers", False),
    (r"msd_final_wide_kernel<2, 2>", "msd_final_tiers", False),
    (r"msd_final_kernel<", "msd_final", False),        # (tables of other widths: in msd_final)
    (r"msd_final_wide_kernel", "msd_final", False),
    (r"msd_part_a_kernel", "msd_part_a", True),
    (r"msd_part_b(_pipe)?_kernel", "msd_part_b", True),
    (r"msd_bases_kernel", "msd_runs", True),
    (r"msd_runs_seg_kernel", "msd_runs", False),
    (r"msd_runs_apply_kernel", "msd_runs", False),
    (r"msd_group_kernel", "msd_group", True),
    (r"msd_group_sum_kernel", "msd_group", False),
    (r"msd_sample_kernel", "msd_sample", True),
    (r"msd_count_scan_kernel", "msd_count_scan", True),
    (r"msd_compact_kernel", "msd_compact", True),
    (r"gen_uniform_kernel", "gen_uniform", True),
    (r"gen_zipf_kernel", "gen_zipf", True),
    (r"gen_wide_kernel", "gen_wide", True),
    (r"msd_part1c?_kernel", "partition_1pass", True),
    (r"msd_p1c_desc_kernel", "partition_1pass", False),
    (r"msd_big_stage_kernel", "msd_big_dev", True),
    (r"msd_giant_\w+_kernel", "msd_big_dev", False),
    (r"msd_single_kernel", "msd_single", True),
]


def tag_of(name):
    for rx, tag, primary in TAGS:
        if re.search(rx, name):
            return tag, primary
    return None, False


def read_counter(d, counter, summary_csv=None):
    """Per-scope counter totals and primary-kernel dispatch counts; with
    summary_csv, also the raw per-kernel totals (every kernel, its dispatch
    count, the counter summed over its dispatches) -- the committed record the
    JSON is computed from."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    total = defaultdict(float)
    launches = defaultdict(int)
    raw = defaultdict(lambda: [0, 0.0])
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                raw[name][0] += 1
                raw[name][1] += float(row["Counter_Value"])
                t, primary = tag_of(name)
                if t:
                    total[t] += float(row["Counter_Value"])
                    launches[t] += primary
    if summary_csv:
        with open(summary_csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["kernel", "dispatches", f"{counter}_kib_total"])
            for name, (n, v) in sorted(raw.items(), key=lambda kv: -kv[1][1]):
                w.writerow([name, n, round(v, 1)])
    return total, launches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--workload", default="c3", help="bench.py --workload the runs timed (c3 / c4 / c5)")
    ap.add_argument("--runs", type=int, default=5,
                    help="bench.py steps the PMC runs executed: warmup + steps + profiling steps (1 + 2 + 2)")
    ap.add_argument("-o", "--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--source-sha", default=None,
                    help="smj._lib.source_sha() of the tree the PMC runs used (default: <fetch_dir>/../source_sha.txt "
                         "written by tools/gpu_run.sh on the box, else this tree's)")
    a = ap.parse_args()
    base = os.path.splitext(a.out)[0]
    fcsv, wcsv = base + "_fetch_summary.csv", base + "_write_summary.csv"
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    fetch, nf = read_counter(a.fetch_dir, "FETCH_SIZE", fcsv)
    write, nw = read_counter(a.write_dir, "WRITE_SIZE", wcsv)
    kernels = {}
    for t in sorted(set(fetch) | set(write)):
        f = fetch.get(t, 0.0) / max(nf.get(t, 0), 1)
        w = write.get(t, 0.0) / max(nw.get(t, 0), 1)
        kernels[t] = {"launches": nf.get(t, 0), "fetch_kib_raw": round(f, 1),
                      "write_kib": round(w, 1), "hbm_bytes_per_launch": round((2 * f + w) * 1024)}
    sha = a.source_sha
    side = os.path.join(os.path.dirname(os.path.normpath(a.fetch_dir)), "source_sha.txt")
    if sha is None and os.path.exists(side):
        sha = open(side).read().strip()
    if sha is None:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "pim-sort-merge-join_amd"))
        from smj._lib import source_sha
        sha = source_sha()
    out = {"rows_per_table": a.rows, "workload": a.workload, "runs": a.runs, "source_sha": sha,
           "source": [fcsv, wcsv],
           "raw_runs": [a.fetch_dir, a.write_dir],
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB per scope launch (gfx950: FETCH_SIZE "
                         "counts half of a wide coalesced read; MI355X_MICROARCH.md, HBM)",
           "kernels": kernels}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for t, k in kernels.items():
        print(f"{t:20s} {k['hbm_bytes_per_launch'] / 1e9:8.3f} GB/launch  ({k['launches']} launches)")


if __name__ == "__main__":
    main()
