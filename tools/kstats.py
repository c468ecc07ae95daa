#!/usr/bin/env python3
"""Print per-kernel average durations from a rocprofv3 --stats CSV (or a rocpd
.db), short names, sorted by total time.  Usage: kstats.py <file> [n]"""
import csv
import sqlite3
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    if "rocprim" in n:
        for key in ("radix_sort", "merge_sort", "scan_impl", "partition", "lookback"):
            if key in n:
                return "rocprim:" + key
    return n.split("(")[0][:70]


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(r[0], int(r[1]), float(r[2])) for r in c.execute("select name, total_calls, total_duration from top_kernels")]
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))]


if __name__ == "__main__":
    agg = {}
    for name, calls, tot in rows(sys.argv[1]):
        k = short(name)
        a = agg.setdefault(k, [0, 0.0])
        a[0] += calls
        a[1] += tot
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    for k, (calls, tot) in sorted(agg.items(), key=lambda x: -x[1][1])[:n]:
        print(f"{tot / 1e6:10.3f} ms total {calls:6d} calls {tot / calls / 1e6:9.4f} ms avg  {k}")
