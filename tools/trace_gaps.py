"""GPU idle gaps in a rocprofv3 kernel trace (…_kernel_trace.csv).

    python tools/trace_gaps.py TRACE.csv [--top 25] [--from-kernel NAME]

Prints the union of kernel busy time against the wall span of the trace
(from the first launch of --from-kernel, if given), the busy time per kernel
name, and the largest idle gaps with the kernels on either side: where a
step's time goes outside any kernel (host synchronisations, launch gaps).
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--from-kernel", default=None)
    ap.add_argument("--per", default=None, help="also split the trace into windows at each launch of this kernel")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60]))
    rows.sort()
    if a.from_kernel:
        i0 = next(i for i, r in enumerate(rows) if a.from_kernel in r[2])
        rows = rows[i0:]
    busy, gaps, per = 0, [], defaultdict(float)
    cur_s, cur_e, prev = rows[0][0], rows[0][1], rows[0][2]
    for s, e, n in rows:
        per[n] += (e - s) / 1e6
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(((s - cur_e) / 1e6, prev, n, (cur_e - rows[0][0]) / 1e6))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n
    busy += cur_e - cur_s
    wall = (rows[-1][1] - rows[0][0]) / 1e6
    print(f"kernels {len(rows)}  wall {wall:.3f} ms  busy {busy / 1e6:.3f} ms  idle {wall - busy / 1e6:.3f} ms")
    print("busy per kernel (ms, overlaps counted per kernel):")
    for n, t in sorted(per.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  {t:9.3f}  {n}")
    print(f"largest idle gaps (ms, after -> before, at ms):")
    for g, p, n, at in sorted(gaps, reverse=True)[: a.top]:
        print(f"  {g:8.3f}  {p} -> {n}  @{at:.3f}")
    if a.per:
        # per window (from one launch of --per to the next): idle time, and the
        # idle summed per (kernel before, kernel after) pair over all windows
        starts = [r[0] for r in rows if a.per in r[2]] + [rows[-1][1] + 1]
        t0 = rows[0][0]
        pairs = defaultdict(lambda: [0.0, 0])
        print(f"windows at {a.per}: start ms, wall ms, idle ms")
        for w0, w1 in zip(starts[:-1], starts[1:]):
            gs = [g for g in gaps if w0 <= t0 + g[3] * 1e6 < w1]
            idle = sum(g[0] for g in gs)
            last = max(r[1] for r in rows if w0 <= r[0] < w1)
            print(f"  {(w0 - t0) / 1e6:9.3f}  {(last - w0) / 1e6:8.3f}  {idle:7.3f}")
            for g in gs:
                pairs[(g[1], g[2])][0] += g[0]
                pairs[(g[1], g[2])][1] += 1
        print("idle per kernel pair over the windows (ms, gaps):")
        for (p, n), (t, c) in sorted(pairs.items(), key=lambda kv: -kv[1][0])[:20]:
            print(f"  {t:8.3f} {c:5d}  {p} -> {n}")


if __name__ == "__main__":
    main()
