"""One step of a rocprofv3 kernel trace as a timeline: every kernel over
--min-ms (or after an idle gap over --min-gap ms) with its start / end in ms
from the step start, its hardware queue and the gap before it.  Steps start
at the --mark kernel (default: the first chunk_hist of a distributed step,
two per step); --step picks which (default: the third, past the warmup).

    python tools/trace_steps.py gpurun_out/r03d/ltrace/loop_kernel_trace.csv
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--mark", default="chunk_hist")
    ap.add_argument("--per-step", type=int, default=2)
    ap.add_argument("--step", type=int, default=2)
    ap.add_argument("--min-ms", type=float, default=0.1)
    ap.add_argument("--min-gap", type=float, default=0.05)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48],
                         r["Queue_Id"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.mark in r[2]][:: a.per_step]
    i0, i1 = marks[a.step], marks[a.step + 1]
    t0 = prev = rows[i0][0]
    busy = 0
    for s, e, n, q in rows[i0:i1]:
        gap = (s - prev) / 1e6
        if (e - s) / 1e6 > a.min_ms or gap > a.min_gap:
            print(f"{(s - t0) / 1e6:8.3f} - {(e - t0) / 1e6:8.3f} ms  queue {q:>2}  gap {gap:6.3f}  {n}")
        prev = max(prev, e)
    print(f"step {a.step}: {(rows[i1][0] - t0) / 1e6:.3f} ms to the next step's first {a.mark}")


if __name__ == "__main__":
    main()
