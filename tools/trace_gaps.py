"""GPU idle time from a rocprofv3 kernel trace: the union of the kernel
intervals against the wall span, and the largest gaps with the kernels around
them (what ran before / after each idle period).

    python tools/trace_gaps.py gpurun_out/<tag>/tr/<name>_kernel_trace.csv [t0_ms t1_ms]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    base = ev[0][0]
    if len(sys.argv) > 3:
        lo, hi = base + float(sys.argv[2]) * 1e6, base + float(sys.argv[3]) * 1e6
        ev = [e for e in ev if e[0] >= lo and e[1] <= hi]
    busy, gaps, end, prev = 0, [], ev[0][0], None
    for s, e, n in ev:
        if s > end:
            gaps.append((s - end, end, prev, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        prev = n
    wall = end - ev[0][0]
    print(f"span {wall / 1e6:.3f} ms, GPU busy {busy / 1e6:.3f} ms ({busy / wall:.1%}), idle {sum(g[0] for g in gaps) / 1e6:.3f} ms "
          f"in {len(gaps)} gaps")
    for g, at, a, b in sorted(gaps, reverse=True)[:15]:
        print(f"  {g / 1e3:8.1f} us at {(at - base) / 1e6:9.3f} ms: after {a[:50]} | before {b[:50]}")


if __name__ == "__main__":
    main()
