#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory into profiles/<tag>/.

Copies the rocprofv3 kernel-stats CSV (the --kernel-trace --stats summary)
and reduces the PMC passes to per-kernel averages (one row per kernel and
counter), adding the gfx950-corrected HBM read traffic of each kernel:
hbm_read_bytes = FETCH_SIZE (KiB) * 1024 * 2  (MI355X_MICROARCH.md §HBM: on
gfx950 FETCH_SIZE reports half the bytes of a 16 B/lane streaming read).

Usage: python tools/prof_summary.py gpurun_out/prof_r01 profiles/r01
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    n = n.split("(")[0]
    return n.split("::")[-1] if "::" in n else n[:80]


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    st = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(dst, "kernel_stats.csv"))
    out = {}
    for sub in sorted(os.listdir(src)):
        fn = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(fn):
            continue
        d = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(fn)):
            k = short(r["Kernel_Name"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            d[k][r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
        for k, cs in d.items():
            e = out.setdefault(k, {})
            for c, l in cs.items():
                e[c] = sum(x for x, _ in l) / len(l)
                e.setdefault("dispatches_" + sub, len(l))
                e["avg_ms_" + sub] = sum(t for _, t in l) / len(l)
            if "FETCH_SIZE" in e:
                e["hbm_read_bytes_corrected"] = e["FETCH_SIZE"] * 1024 * 2
    json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
    # per-launch HBM read traffic of the scan kernel, for bench.py's roofline
    alg = os.environ.get("PROF_ALG_BYTES")
    for k, e in out.items():
        if k.startswith(("k_scan_fast", "k_scan_big")) and "hbm_read_bytes_corrected" in e and alg:
            t = {"kernel": k, "hbm_read_bytes_per_launch": e["hbm_read_bytes_corrected"],
                 "algorithmic_bytes_per_launch": int(alg), "source": os.path.join(dst, "pmc_summary.json"),
                 "note": "FETCH_SIZE KiB x 1024 x 2 (gfx950: FETCH_SIZE reports half of a 16 B/lane stream)"}
            name = "k_scan_big" if k.startswith("k_scan_big") else "k_scan_fast"
            json.dump(t, open(os.path.join(os.path.dirname(dst.rstrip("/")), f"traffic_{name}.json"), "w"), indent=1)
    for k, e in sorted(out.items()):
        print(k, {c: round(v, 3) for c, v in e.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
