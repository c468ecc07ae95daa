#!/usr/bin/env python3
"""Timeline of one bench step from a rocprofv3 --kernel-trace CSV: every
kernel of the step that starts at the last launch of <anchor> (default the
scan kernel), in order, with its start offset, duration and the idle gap
before it -- where the time between kernels goes (host round trips, launch
latency, copies).  Usage: timeline.py <run_kernel_trace.csv> [anchor] [n_before]"""
import csv
import sys

from kstats import short


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_scan_"
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    starts = [i for i, (_, _, n) in enumerate(rows) if n.startswith(anchor)]
    if not starts:
        print("anchor not found")
        return
    # the last step: from `before` kernels ahead of the last anchor launch to the end
    before = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    a = max(0, starts[-1] - before)
    t0 = rows[a][0]
    prev_end = t0
    busy = 0
    print(f"{'start_ms':>9} {'dur_ms':>8} {'gap_ms':>8}  kernel")
    for s, e, n in rows[a:]:
        gap = (s - prev_end) / 1e6
        print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} {gap:8.3f}  {n}")
        busy += e - s
        prev_end = max(prev_end, e)
    print(f"span {(prev_end - t0) / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
