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


CUS, SIMDS, XCDS = 256, 1024, 8


def derive(e):
    """Derived per-dispatch metrics (keys prefixed `d_`), each from counters
    of ONE pass (tools/pmc.sh) and that pass's own average duration:
    * d_lds_bank_conflict_rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
      (extra conflict cycles over all LDS-array cycles)
    * d_valu_per_lds = SQ_INSTS_VALU / SQ_INSTS_LDS
    * d_clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / duration
    * d_valu_busy = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (1024 SIMDs x
      GRBM_GUI_ACTIVE / 8): share of SIMD cycles issuing VALU
    * d_lds_busy, d_issue_busy: the same for SQ_ACTIVE_INST_LDS / _ANY
    * d_waves_per_simd = SQ_WAVE_CYCLES x 4 / (1024 SIMDs x cycles), cycles
      from the sq pass's duration at the busy pass's clock (occupancy)
    * d_hbm_read_GBps = FETCH_SIZE x 2 KiB / duration of the fetch pass"""
    g = e.get("GRBM_GUI_ACTIVE")
    if e.get("SQ_LDS_IDX_ACTIVE"):
        e["d_lds_bank_conflict_rate"] = e.get("SQ_LDS_BANK_CONFLICT", 0.0) / e["SQ_LDS_IDX_ACTIVE"]
    if e.get("SQ_INSTS_LDS"):
        e["d_valu_per_lds"] = e.get("SQ_INSTS_VALU", 0.0) / e["SQ_INSTS_LDS"]
    if g and e.get("avg_ms_busy"):
        cyc = g / XCDS
        e["d_clock_ghz"] = cyc / (e["avg_ms_busy"] * 1e6)
        for c, n in (("SQ_ACTIVE_INST_VALU", "d_valu_busy"), ("SQ_ACTIVE_INST_LDS", "d_lds_busy"),
                     ("SQ_ACTIVE_INST_ANY", "d_issue_busy")):
            if c in e:
                e[n] = e[c] * 4 / (SIMDS * cyc)
        if "SQ_WAVE_CYCLES" in e and e.get("avg_ms_sq"):
            e["d_waves_per_simd"] = e["SQ_WAVE_CYCLES"] * 4 / (SIMDS * e["d_clock_ghz"] * e["avg_ms_sq"] * 1e6)
    if "FETCH_SIZE" in e and e.get("avg_ms_fetch"):
        e["d_hbm_read_GBps"] = e["FETCH_SIZE"] * 2048 / (e["avg_ms_fetch"] * 1e6)


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
    for k, e in out.items():
        derive(e)
    json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
    # per-launch HBM read traffic of the scan kernel, for bench.py's roofline
    alg = os.environ.get("PROF_ALG_BYTES")
    for k, e in out.items():
        if k.startswith(("k_scan_fast", "k_scan_big", "k_scan_lines")) and "hbm_read_bytes_corrected" in e and alg:
            t = {"kernel": k, "hbm_read_bytes_per_launch": e["hbm_read_bytes_corrected"],
                 "algorithmic_bytes_per_launch": int(alg), "source": os.path.join(dst, "pmc_summary.json"),
                 "note": "FETCH_SIZE KiB x 1024 x 2 (gfx950: FETCH_SIZE reports half of a 16 B/lane stream)"}
            name = k.split("<")[0]
            json.dump(t, open(os.path.join(os.path.dirname(dst.rstrip("/")), f"traffic_{name}.json"), "w"), indent=1)
    for k, e in sorted(out.items()):
        print(k, {c: round(v, 3) for c, v in e.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
