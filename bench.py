#!/usr/bin/env python3
"""bench.py — Trivy secret-scan throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): full builtin ruleset (keyword prefilter +
regex verification + line numbers + allow rules) over a synthetic mixed-text
corpus resident in HBM, secrets planted at 1e-6 per byte.  Default 50 GB per
GPU; one step = one complete Scanner.Scan pass over every file of the shard
(tsg_scan_device).  Multi-GPU: one process per GPU, each scanning its own
shard (independent files: no data-path collective) -> weak scaling.

Other BASELINE configs (`--config N`, extra measurement lines, not the
headline): 1 = keyword prefilter only (tsg_gate_device, 20 GB), 4 = stress:
builtin + 1000 generated gitleaks-style custom rules (tests/stress_rules.py;
the automaton no longer fits k_scan_fast's LDS image).

Prints ONE JSON line (rank 0).  Roofline is reported for the dominant kernel
(k_scan, the HBM pass).  cpu_baseline times bench_cpu/cpu_scan.cpp (the Go
scanner's Scan restated in C++ on the repo's host Go-regexp VM, multi-threaded;
Go is not installed) on a bounded sample of the same corpus.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PLANT_DTYPE = np.dtype([("file", "<u4"), ("tpl", "<u4"), ("start", "<u8"), ("end", "<u8"),
                        ("decoy", "<u4"), ("pad", "<u4")])
# plant kinds (corpus.hip PlantKind): 0 real, 1 one-char-short decoy, 2 EXAMPLE decoy, 3 K/ſ-spelled instance
PLANT_REAL, PLANT_SHORT, PLANT_EXAMPLE, PLANT_FOLD = 0, 1, 2, 3
WORKLOADS = {
    0: "configs[0]: builtin rules through the batched SecretAnalyzer (IsBinary, CR strip, scan, findings) on a "
       "1 GB source tree already read into host memory; PCIe-inclusive (pinned staging + H2D in the step)",
    1: "configs[1]: keyword prefilter only (Aho-Corasick over all builtin rule keywords, per-file rule gates), "
       "mixed text corpus resident in HBM",
    2: "configs[2]: full builtin ruleset (prefilter + regex + line numbers + allow rules), mixed text corpus "
       "resident in HBM",
    3: "configs[3]: image-layer set, builtin rules: one layer tar per GPU in host memory (ustar members = the "
       "SURVEY.md §8(d) corpus files), native layer walk (whiteouts, skip rules) + SecretAnalyzer.Required + one "
       "batched analyze (IsBinary, CR strip, scan, findings) per layer; PCIe-inclusive (pinned staging + H2D in "
       "the step); file shards = layers per rank",
    4: "configs[4]: stress, builtin + generated gitleaks-style custom rules (explosion rules, keyword-less rules), "
       "mixed text corpus resident in HBM + 2 % C5 material (stress-rule instances, 16 MiB minified line, "
       "binary-ish files)",
}
HBM_PEAK_GBPS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md


def file_sizes(seed, target_bytes):
    """Lognormal sizes, median 6 KiB, sigma 1.6, clipped to [10 B, 64 MiB]."""
    rng = np.random.default_rng(seed)
    sizes = []
    total = 0
    while total < target_bytes:
        s = np.clip(rng.lognormal(np.log(6144.0), 1.6, 1 << 20), 10, 64 << 20).astype(np.int64)
        c = np.cumsum(s)
        k = int(np.searchsorted(c, target_bytes - total)) + 1
        sizes.append(s[:k])
        total += int(s[:k].sum())
    return np.concatenate(sizes)


def build_corpus(N, torch, seed, gb, density, device):
    sizes = file_sizes(seed, int(gb * 1e9))
    n_files = len(sizes)
    # device layout (include/trivy_secret_gpu.h): each file followed by one NUL separator
    off = np.zeros(n_files + 1, dtype=np.uint64)
    off[1:] = np.cumsum(sizes + 1).astype(np.uint64)
    total = int(off[-1])
    content = int(sizes.sum())
    chunk = N.gen.tsg_gen_chunk_bytes()
    nchunks = (sizes + chunk - 1) // chunk
    file_of = np.repeat(np.arange(n_files, dtype=np.uint64), nchunks)
    first = np.repeat(np.cumsum(nchunks) - nchunks, nchunks)
    cidx = np.arange(len(file_of), dtype=np.uint64) - first.astype(np.uint64)
    chunk_ids = (file_of << np.uint64(24)) | cidx
    dev = torch.device("cuda", device)
    d_data = torch.zeros(total + 4096, dtype=torch.uint8, device=dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_chunks = torch.from_numpy(chunk_ids.view(np.int64)).to(dev)
    d_paths = torch.empty(n_files * 31 + 64, dtype=torch.uint8, device=dev)
    d_poff = torch.empty(n_files + 1, dtype=torch.int64, device=dev)
    plant_cap = max(1 << 16, int(total * density * 4) + 1024)
    rec = N.gen.tsg_gen_plant_record_size()
    assert rec == PLANT_DTYPE.itemsize
    d_plants = torch.empty(plant_cap * rec, dtype=torch.uint8, device=dev)
    d_np = torch.zeros(1, dtype=torch.int64, device=dev)
    N.check(N.gen.tsg_gen_corpus_device(
        ctypes.c_void_p(d_data.data_ptr()), ctypes.c_void_p(d_off.data_ptr()), ctypes.c_void_p(d_chunks.data_ptr()),
        len(chunk_ids), ctypes.c_void_p(d_paths.data_ptr()), ctypes.c_void_p(d_poff.data_ptr()), n_files,
        seed, density, ctypes.c_void_p(d_plants.data_ptr()), plant_cap, ctypes.c_void_p(d_np.data_ptr())))
    nplants = min(int(d_np.item()), plant_cap)
    plants = np.frombuffer(d_plants[: nplants * rec].cpu().numpy().tobytes(), dtype=PLANT_DTYPE)
    del d_chunks
    return dict(n_files=n_files, total=content, packed=total, off=off, d_data=d_data, d_off=d_off, d_paths=d_paths,
                d_poff=d_poff, plants=plants, sizes=sizes)


def stress_material(stress_rules, srules, seed, target_bytes):
    """configs[4] C5 material: stress-rule corpus files (planted custom-rule
    instances), one 16 MiB minified single-line file, binary-ish files; the
    unique set is replicated under new paths up to target_bytes.  Returns
    (unique files, all files) as (path bytes, content bytes)."""
    files = stress_rules.make_corpus(seed + 44, srules, 3000, long_line_bytes=1 << 20)
    big = stress_rules.make_corpus(seed + 45, srules, 0, long_line_bytes=16 << 20)[0]
    uniq = [(p.encode(), d) for p, d in files] + [(b"stress/min/vendor.bundle.min.js", big[1])]
    out, total, k = [], 0, 0
    while total < target_bytes:
        for p, d in uniq:
            out.append((p if k == 0 else b"r%d/" % k + p, d))
            total += len(d)
        k += 1
    return uniq, out


def append_files(torch, c, files, device):
    """The corpus dict with `files` appended (same layout: NUL after each
    file, path offsets continuing), new device tensors."""
    dev = torch.device("cuda", device)
    n0 = c["n_files"]
    sizes = np.array([len(d) for _, d in files], dtype=np.int64)
    off_new = np.zeros(len(files) + 1, dtype=np.uint64)
    off_new[1:] = np.cumsum(sizes + 1).astype(np.uint64)
    blob = np.zeros(int(off_new[-1]), dtype=np.uint8)
    for (_, d), o in zip(files, off_new[:-1]):
        blob[int(o):int(o) + len(d)] = np.frombuffer(d, dtype=np.uint8)
    packed = c["packed"]
    d_data = torch.zeros(packed + len(blob) + 4096, dtype=torch.uint8, device=dev)
    d_data[:packed] = c["d_data"][:packed]
    d_data[packed:packed + len(blob)] = torch.from_numpy(blob).to(dev)
    off = np.concatenate([c["off"], c["off"][-1] + off_new[1:]])
    poff_old = c["d_poff"].cpu().numpy()
    pb = b"".join(p for p, _ in files)
    plen = np.array([len(p) for p, _ in files], dtype=np.int64)
    poff_new = poff_old[-1] + np.concatenate([[0], np.cumsum(plen)])
    d_paths = torch.zeros(int(poff_new[-1]) + 64, dtype=torch.uint8, device=dev)
    d_paths[: int(poff_old[-1])] = c["d_paths"][: int(poff_old[-1])]
    d_paths[int(poff_old[-1]): int(poff_new[-1])] = torch.from_numpy(np.frombuffer(pb, dtype=np.uint8).copy()).to(dev)
    poff = np.concatenate([poff_old, poff_new[1:]]).astype(np.int64)
    c2 = dict(c)
    c2.update(n_files=n0 + len(files), total=c["total"] + int(sizes.sum()), packed=packed + len(blob), off=off,
              d_data=d_data, d_off=torch.from_numpy(off.view(np.int64)).to(dev), d_paths=d_paths,
              d_poff=torch.from_numpy(poff).to(dev), sizes=np.concatenate([c["sizes"], sizes]),
              first_stress=n0)
    return c2


def stress_checks(N, res, rules, c, uniq, oracle_cfg, n_check=80):
    """Oracle spot checks of the appended stress files (full findings, Match
    and Code included), the minified 16 MiB line excluded (oracle time)."""
    from oracle import secret_oracle as O

    oracle = O.Scanner(O.parse_config(oracle_cfg))
    f0 = c["first_stress"]
    bad, found, custom = [], 0, 0
    picks = list(range(0, len(uniq) - 1, max(1, (len(uniq) - 1) // n_check)))[:n_check]
    # binary-ish files in; the minified files (1 and 16 MiB single lines with
    # thousands of findings, each Code line the whole line) only through the
    # GPU tests' smaller minified files -- the oracle would hold GBs of strings
    picks += [i for i, (p, _) in enumerate(uniq) if b"/bin/" in p]
    for i in sorted(set(picks)):
        p, d = uniq[i]
        want = oracle.scan(p.decode(), d)
        found += len(want["Findings"])
        custom += sum(x.RuleID.startswith("stress-") for x in want["Findings"])
        if sorted(result_findings(N, res, f0 + i, rules)) != sorted(oracle_findings(want)):
            bad.append(p.decode())
    return dict(stress_files=len(set(picks)), stress_findings=found, stress_custom_findings=custom,
                stress_mismatched=bad[:10], stress_mismatched_files=len(bad),
                stress_bytes=int(sum(c["sizes"][c["first_stress"]:])))


def build_layer_tar(host, off, sizes, pbytes, poff):
    """The corpus as one ustar layer: a 512-byte header per file (name, mode
    0644, octal size, checksum, typeflag '0'), content padded to 512, two zero
    blocks.  Headers are built vectorised in chunks; content copied per file."""
    n = len(sizes)
    sizes = sizes.astype(np.int64)
    span = 512 + ((sizes + 511) // 512) * 512
    toff = np.zeros(n + 1, dtype=np.int64)
    toff[1:] = np.cumsum(span)
    out = np.zeros(int(toff[-1]) + 1024, dtype=np.uint8)
    plen = np.diff(poff.astype(np.int64))
    assert plen.max() < 100
    step = 1 << 15
    for a in range(0, n, step):
        b = min(n, a + step)
        k = b - a
        H = np.zeros((k, 512), dtype=np.uint8)
        L = plen[a:b]
        rows = np.repeat(np.arange(k), L)
        cols = np.arange(int(L.sum())) - np.repeat(np.cumsum(L) - L, L)
        H[rows, cols] = pbytes[int(poff[a]):int(poff[b])]
        for fo, txt in ((100, b"0000644"), (108, b"0000000"), (116, b"0000000"), (136, b"00000000000"),
                        (148, b"        "), (257, b"ustar\x0000"), (156, b"0")):
            H[:, fo:fo + len(txt)] = np.frombuffer(txt, dtype=np.uint8)
        sz = sizes[a:b]
        for d in range(11):
            H[:, 124 + d] = 48 + ((sz >> (3 * (10 - d))) & 7)
        ck = H.astype(np.int64).sum(axis=1)
        for d in range(6):
            H[:, 148 + d] = 48 + ((ck >> (3 * (5 - d))) & 7)
        H[:, 154] = 0
        H[:, 155] = 32
        out[(toff[a:b, None] + np.arange(512)).ravel()] = H.ravel()
    for i in range(n):
        o, z, t = int(off[i]), int(sizes[i]), int(toff[i]) + 512
        out[t:t + z] = host[o:o + z]
    return out


def shared_layer_set(seed, gb_total, n_layers):
    """configs[3] shared list: the byte sizes of an image's `n_layers` layers
    (lognormal around the mean, sigma 0.6, scaled to gb_total), the same on
    every rank; layer k's files come from seed + 7919 k, so a layer's content
    does not depend on which rank builds it."""
    rng = np.random.default_rng(seed + 77)
    w = rng.lognormal(0.0, 0.6, n_layers)
    return [max(0.002, gb_total * x / w.sum()) for x in w]


def scan_device(N, eng, rs, c):
    res = ctypes.c_void_p()
    N.check(N.lib.tsg_scan_device(eng, rs, ctypes.c_void_p(c["d_data"].data_ptr()),
                                  ctypes.c_void_p(c["d_off"].data_ptr()), ctypes.c_void_p(c["d_paths"].data_ptr()),
                                  ctypes.c_void_p(c["d_poff"].data_ptr()), c["n_files"], ctypes.byref(res)))
    return res


def result_timings(N, res):
    tm = (ctypes.c_double * 32)()
    nt = ctypes.c_size_t()
    N.lib.tsg_result_timings(res, tm, 32, ctypes.byref(nt))
    return [tm[i] for i in range(min(32, nt.value))]


def read_result(N, res):
    n = N.lib.tsg_result_loc_count(res)
    locs = N.lib.tsg_result_locs(res)
    arr = np.ctypeslib.as_array(ctypes.cast(locs, ctypes.POINTER(ctypes.c_uint8)),
                                shape=(n * ctypes.sizeof(N.LocC),)).copy() if n else np.zeros(0, np.uint8)
    dt = np.dtype([("file", "<u4"), ("rule", "<u4"), ("start", "<u8"), ("end", "<u8"),
                   ("start_line", "<u4"), ("end_line", "<u4")])
    locs = np.frombuffer(arr.tobytes(), dtype=dt)
    tm = (ctypes.c_double * 32)()
    nt = ctypes.c_size_t()
    N.lib.tsg_result_timings(res, tm, 32, ctypes.byref(nt))
    return locs, [tm[i] for i in range(min(32, nt.value))]


def template_rules(N):
    """Rule ID of each corpus.hip template (one per builtin rule)."""
    return [N.gen.tsg_gen_template_rule(i).decode() for i in range(N.gen.tsg_gen_template_count())]


def result_findings(N, res, f, rules):
    """Findings of file f from a result (device-built Match / Code), in order."""
    fp = ctypes.POINTER(N.FindingC)()
    k = N.lib.tsg_result_findings(res, f, ctypes.byref(fp))
    out = []
    for j in range(k):
        x = fp[j]
        lines = tuple((x.lines[q].number, ctypes.string_at(x.lines[q].content, x.lines[q].content_len),
                       bool(x.lines[q].is_cause), bool(x.lines[q].first_cause), bool(x.lines[q].last_cause))
                      for q in range(x.n_lines))
        out.append((rules[x.rule].id, x.start_line, x.end_line, ctypes.string_at(x.match, x.match_len), lines))
    return out


def oracle_findings(want):
    enc = lambda t: t.encode("utf-8", "surrogateescape")
    return [(x.RuleID, x.StartLine, x.EndLine, enc(x.Match),
             tuple((ln["Number"], enc(ln["Content"]), ln["IsCause"], ln["FirstCause"], ln["LastCause"])
                   for ln in x.Code["Lines"]))
            for x in want["Findings"]]


def parity_checks(N, S, c, locs, rules, seed, density, n_sample=300, oracle_cfg=None, big_files=3,
                  nonascii_files=24, res=None):
    """Full-size properties + oracle spot checks on sample files.

    Properties over the WHOLE batch: every real plant (an instance of one of
    the 86 builtin rules) is reported at its exact location; no decoy (one
    char short, or EXAMPLE inside the match) is.  Spot checks: the oracle's
    Scan of sample files (plant files, random files, `big_files` files of
    4-16 MiB and `nonascii_files` of the 0.1 % carrying é/K/ſ/İ, the K/ſ-spelled
    rule instances first) must equal the engine's locations exactly."""
    from oracle import secret_oracle as O

    tpl_rules = template_rules(N)
    rid = {r.id: i for i, r in enumerate(rules)}
    have = set(zip(locs["file"].tolist(), locs["rule"].tolist(), locs["start"].tolist(), locs["end"].tolist()))
    plants = c["plants"]
    key = lambda p, d=0: (int(p["file"]), rid[tpl_rules[p["tpl"]]], int(p["start"]), int(p["end"]) - d)
    real = plants[plants["decoy"] == PLANT_REAL]
    found = sum(key(p) in have for p in real)
    decoys = plants[(plants["decoy"] == PLANT_SHORT) | (plants["decoy"] == PLANT_EXAMPLE)]
    decoy_hits = sum(key(p) in have or key(p, 1) in have for p in decoys)
    per_rule = {}
    for p in real:
        per_rule[tpl_rules[p["tpl"]]] = per_rule.get(tpl_rules[p["tpl"]], 0) + 1
    # oracle spot checks
    rng = np.random.default_rng(seed + 7)
    sizes = c["sizes"]
    n_gen = c.get("first_stress", c["n_files"])  # generated files (configs[4] appends stress files after them)
    fold = plants[plants["decoy"] == PLANT_FOLD]
    fold_files = [int(f) for f in np.unique(fold["file"]) if sizes[f] <= (8 << 20)]
    nonascii = [f for f in range(n_gen) if sizes[f] >= 600 and N.gen.tsg_gen_file_nonascii(seed, f)]
    extra_na = [f for f in nonascii if f not in set(fold_files) and sizes[f] <= (8 << 20)]
    na_pick = (fold_files + [int(x) for x in rng.permutation(extra_na)])[:nonascii_files]
    big = np.nonzero((sizes[:n_gen] >= (4 << 20)) & (sizes[:n_gen] <= (16 << 20)))[0]
    big_pick = [int(x) for x in rng.permutation(big)[:big_files]]
    cand = np.unique(np.concatenate([real["file"][: n_sample // 2].astype(np.int64),
                                     rng.integers(0, n_gen, n_sample // 2)]))
    cand = sorted(set(int(f) for f in cand if sizes[f] <= (4 << 20)) | set(na_pick) | set(big_pick))
    by_file = {}
    for L in locs:
        by_file.setdefault(int(L["file"]), []).append(
            (rules[int(L["rule"])].id, int(L["start"]), int(L["end"]), int(L["start_line"]), int(L["end_line"])))
    oracle = O.Scanner(O.parse_config(oracle_cfg) if oracle_cfg else None)
    mismatched = []
    spot_findings = spot_bytes = 0
    for f in cand:
        n = int(sizes[f])
        buf = (ctypes.c_uint8 * max(1, n))()
        N.check(N.gen.tsg_gen_file(seed, f, n, density, buf))
        data = bytes(buf)[:n]
        path = bytes(c["d_paths"][f * 31:(f + 1) * 31].cpu().numpy()).decode()
        want = oracle.scan(path, data, with_offsets=True)
        w = sorted((x.RuleID, x.Start, x.End, x.StartLine, x.EndLine) for x in want["Findings"])
        g = sorted(by_file.get(f, []))
        spot_findings += len(w)
        spot_bytes += n
        # the device-built findings in Scan order (Match and Code lines included);
        # (RuleID, Match) ties are order-free in the reference's sort
        full_ok = res is None or sorted(result_findings(N, res, f, rules)) == sorted(oracle_findings(want))
        if res is not None:
            got_ids = [x[0] for x in result_findings(N, res, f, rules)]
            full_ok = full_ok and got_ids == sorted(got_ids)
        if w != g or not full_ok:
            mismatched.append(f)
    return dict(planted=int(len(real)), planted_found=int(found), planted_rules=len(per_rule),
                decoys=int(len(decoys)), decoys_found=int(decoy_hits), fold_instances=int(len(fold)),
                nonascii_files=len(nonascii), spot_files=len(cand), spot_bytes=spot_bytes,
                spot_nonascii_files=len(na_pick), spot_big_files=len(big_pick),
                spot_max_file_bytes=int(max(sizes[f] for f in cand)) if cand else 0,
                spot_findings=spot_findings, spot_mismatched_files=len(mismatched),
                spot_mismatched=mismatched[:10], total_findings=int(len(locs)))


def gate_timings(N, eng):
    """Timings of the engine's last tsg_gate_device call (tsg_engine_gate_timings)."""
    tm = (ctypes.c_double * 32)()
    nt = ctypes.c_size_t()
    N.check(N.lib.tsg_engine_gate_timings(eng, tm, 32, ctypes.byref(nt)))
    return [tm[i] for i in range(min(32, nt.value))]


def gate_checks(N, c, rules, gates, words, seed, density, n_sample=200):
    """configs[1] parity: gate bits of sample files against the oracle's MatchKeywords."""
    from oracle import secret_oracle as O

    g = np.frombuffer(bytes(gates), dtype=np.uint32).reshape(c["n_files"], words)
    orules = O.Scanner(None).rules
    rng = np.random.default_rng(seed + 9)
    cand = [int(f) for f in np.unique(rng.integers(0, c["n_files"], n_sample)) if c["sizes"][f] <= (4 << 20)]
    bad = 0
    passed = 0
    for f in cand:
        n = int(c["sizes"][f])
        buf = (ctypes.c_uint8 * max(1, n))()
        N.check(N.gen.tsg_gen_file(seed, f, n, density, buf))
        data = bytes(buf)[:n]
        low = O.go_bytes_to_lower(data)
        want = [O.Scanner.match_keywords(r, data, low) for r in orules]
        got = [bool((g[f, i // 32] >> (i % 32)) & 1) for i in range(len(rules))]
        passed += sum(want)
        bad += want != got
    return dict(spot_files=len(cand), spot_gate_bits_set=passed, spot_mismatched_files=bad,
                files_with_any_keyword_rule=int(sum(bool(x.any()) for x in g)))


def traffic_bytes(content_bytes, kernel="k_scan_fast"):
    """HBM bytes per k_scan_fast launch from the committed rocprofv3 FETCH_SIZE
    pass (profiles/traffic_k_scan_fast.json, written by tools/prof_summary.py:
    FETCH_SIZE KiB x 1024 x 2, the gfx950 correction), scaled to this launch's
    content bytes when the profiled corpus differs.  None without a profile."""
    p = os.path.join(ROOT, "profiles", f"traffic_{kernel}.json")
    if not os.path.exists(p):
        return None, None
    t = json.load(open(p))
    return round(t["hbm_read_bytes_per_launch"] * content_bytes / t["algorithmic_bytes_per_launch"]), t["source"]


def physical_cores():
    """Physical cores of this host (unique (package, core) pairs in /proc/cpuinfo)."""
    pairs, phys, core = set(), None, None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
            elif not line.strip() and core is not None:
                pairs.add((phys, core))
                core = None
    except OSError:
        pass
    return len(pairs) or None


def cpu_quota():
    """CPUs this process may actually use: the affinity set, capped by the
    cgroup CPU quota (cpu.max / cfs_quota_us) -- on the GPU box the affinity set
    lists the whole machine while the quota is the box's share, and threads
    beyond the quota only time-slice."""
    n = len(os.sched_getaffinity(0))
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            parts = open(path).read().split()
        except OSError:
            continue
        if path.endswith("cpu.max"):
            if parts and parts[0] != "max":
                n = min(n, max(1, -(-int(parts[0]) // int(parts[1]))))
        else:
            q = int(parts[0])
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                n = min(n, max(1, -(-q // period)))
        break
    return n


def cpu_lib():
    """bench_cpu/libtsg_cpu_scan.so: Scanner.Scan restated in C++ on the repo's
    host Go-regexp VM (tsgb_cpu_scan), and per-file finding digests of an engine
    result read through the drop-in ABI (tsgb_result_digest): tests/digest.py."""
    lib = ctypes.CDLL(os.path.join(ROOT, "bench_cpu", "libtsg_cpu_scan.so"))
    lib.tsgb_cpu_scan.restype = ctypes.c_int
    lib.tsgb_cpu_scan.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]
    lib.tsgb_result_digest.restype = ctypes.c_int
    lib.tsgb_result_digest.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.c_void_p, ctypes.c_void_p]
    return lib


def gpu_digests(N, lib, res, n_files):
    """(count, digest) per file of an engine result: every finding's rule,
    location, StartLine, EndLine, Match and Code lines (tsg_result_findings)."""
    cnt = np.zeros(n_files, dtype=np.uint32)
    dig = np.zeros(n_files, dtype=np.uint64)
    fn = ctypes.cast(N.lib.tsg_result_findings, ctypes.c_void_p)
    N.check(lib.tsgb_result_digest(fn, res, 0, n_files, cnt.ctypes.data, dig.ctypes.data))
    return cnt, dig


def cpu_scan_range(N, lib, c, a, b, threads):
    """tsgb_cpu_scan over files [a, b) of the corpus, copied from HBM (copy not
    timed): (content bytes, wall seconds, per-file counts, per-file digests)."""
    off = c["off"]
    poff = c["poff_host"]
    host = c["d_data"][int(off[a]): int(off[b])].cpu().numpy()
    pb = c["d_paths"][int(poff[a]): int(poff[b])].cpu().numpy().tobytes()
    p0 = int(poff[a])
    paths = [pb[int(poff[i]) - p0:int(poff[i + 1]) - p0] for i in range(a, b)]
    arr = (ctypes.c_char_p * (b - a))(*paths)
    loff = (off[a:b + 1] - off[a]).astype(np.uint64)
    per = np.zeros(b - a, dtype=np.uint32)
    dig = np.zeros(b - a, dtype=np.uint64)
    tot, sec = ctypes.c_uint64(), ctypes.c_double()
    N.check(lib.tsgb_cpu_scan(c["rs_handle"], host.ctypes.data, loff.ctypes.data, b - a,
                              ctypes.cast(arr, ctypes.c_void_p), threads, 0, per.ctypes.data, dig.ctypes.data,
                              ctypes.byref(tot), ctypes.byref(sec)))
    return int(off[b] - off[a]) - (b - a), sec.value, per, dig


def cpu_baseline(N, c, res, seconds, threads):
    """Time bench_cpu/libtsg_cpu_scan.so — Scanner.Scan restated in C++ on
    the repo's host Go-regexp VM, `threads` threads — on a bounded sample of the
    same corpus: the first files in index order, copied from HBM (copy excluded
    from the clock).  Every sampled file's complete findings (digest of rule,
    location, lines, Match, Code) are compared with the GPU run's."""
    lib = cpu_lib()
    off = c["off"]
    g_cnt, g_dig = gpu_digests(N, lib, res, c["n_files"])
    # calibrate on ~64 MB, then size the sample for `seconds` of wall time
    k0 = max(1, min(int(np.searchsorted(off, 64 << 20)), c["n_files"]))
    b0, t0, _, _ = cpu_scan_range(N, lib, c, 0, k0, threads)
    want = min(int(b0 / max(t0, 1e-6) * seconds), 16 << 30, int(off[-1]))
    k = max(k0, min(c["n_files"], int(np.searchsorted(off, want))))
    nbytes, dt, per, dig = cpu_scan_range(N, lib, c, 0, k, threads)
    same = (per == g_cnt[:k]) & (dig == g_dig[:k])
    phys = physical_cores()
    return dict(value=nbytes / dt / 1e9, unit="GB/s", cores=threads, kind="cpp-restatement",
                physical_cores=phys,
                sample=f"{k} files / {nbytes / 1e6:.1f} MB of the same corpus (first files in index order, copied "
                       f"from HBM), {dt:.1f}s wall on {threads} threads (every CPU this process may use: its affinity "
                       f"set of {len(os.sched_getaffinity(0))} capped by the cgroup CPU quota"
                       + (f"; the host has {phys} physical cores" if phys else "") + "); "
                       "bench_cpu/cpu_scan.cpp: Scanner.Scan restated in C++ on the repo's host Go-regexp VM "
                       "(not Go: no Go toolchain in the image); complete findings (rule, offsets, lines, Match, "
                       f"Code) identical to the GPU's on {int(same.sum())}/{k} files",
                files_identical=int(same.sum()), files=k, findings=int(per.sum()))


def full_parity(N, c, res, threads, ranges, label):
    """Every file of `ranges` ([a, b) file index ranges) through the C++
    restatement (pinned to the oracle by tests/test_cpu_baseline.py), its
    complete findings compared with the GPU result's, file by file.  Chunks of
    ~4 GB; a progress line per chunk on stderr."""
    lib = cpu_lib()
    g_cnt, g_dig = gpu_digests(N, lib, res, c["n_files"])
    off = c["off"]
    files = same = nbytes = f_cpu = f_gpu = 0
    secs = 0.0
    bad = []
    t_all = time.perf_counter()
    for a, b in ranges:
        while a < b:
            e = int(np.searchsorted(off, off[a] + (4 << 30), side="right")) - 1
            e = min(b, max(a + 1, e))
            nb, dt, per, dig = cpu_scan_range(N, lib, c, a, e, threads)
            ok = (per == g_cnt[a:e]) & (dig == g_dig[a:e])
            bad += [a + int(i) for i in np.nonzero(~ok)[0][:10]]
            files += e - a
            same += int(ok.sum())
            nbytes += nb
            secs += dt
            f_cpu += int(per.sum())
            f_gpu += int(g_cnt[a:e].sum())
            print(f"full parity [{label}] files {a}..{e}: {same}/{files} identical, {nbytes / 1e9:.2f} GB, "
                  f"cpu {secs:.0f}s", file=sys.stderr, flush=True)
            a = e
    return dict(files=files, files_identical=same, mismatched=bad[:10], bytes=nbytes, findings_cpu=f_cpu,
                findings_gpu=f_gpu, cpu_seconds=round(secs, 1), wall_seconds=round(time.perf_counter() - t_all, 1),
                threads=threads, scope=label)


_ORACLE_W = {}


def _oracle_worker_init(gen_path, seed, density):
    """A worker of oracle_parity: the bench corpus generator (host side of
    bench_gen/corpus.hip, regenerating each file from its seed) and the
    Python oracle's Scanner (the independent checker: its own regex engine)."""
    from oracle import secret_oracle as O

    gen = ctypes.CDLL(gen_path)
    gen.tsg_gen_file.restype = ctypes.c_int
    gen.tsg_gen_file.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p]
    _ORACLE_W.update(gen=gen, seed=seed, density=density, scanner=O.Scanner(None))


def _oracle_worker(item):
    f, n, path = item
    w = _ORACLE_W
    buf = (ctypes.c_uint8 * max(1, n))()
    rc = w["gen"].tsg_gen_file(w["seed"], f, n, w["density"], buf)
    if rc:
        raise RuntimeError(f"tsg_gen_file({f}) failed: {rc}")
    want = w["scanner"].scan(path, bytes(buf)[:n])
    return f, sorted(oracle_findings(want))


def oracle_parity(N, c, res, rules, seed, density, random_gb, workers):
    """Independent full-size parity: the Python oracle --
    not the C++ restatement, which shares the engine's Go-RE2 parser and VM --
    over every configs[2] file that holds a plant or a decoy, every file the
    GPU reported a finding in, every non-ASCII file (é / K / ſ / İ), and
    random files up to `random_gb`, each regenerated on the host from the
    corpus seed in `workers` processes; complete findings (RuleID, lines,
    Match, every Code line with its flags) compared with the GPU result's."""
    import multiprocessing as mp

    t0 = time.perf_counter()
    sizes = c["sizes"]
    n_gen = c.get("first_stress", c["n_files"])
    locs, _ = read_result(N, res)
    plants = c["plants"]
    pick = set(int(f) for f in np.unique(plants["file"]))
    n_plant = len(pick)
    gpu_files = set(int(f) for f in np.unique(locs["file"]))
    pick |= gpu_files
    nonascii = [f for f in range(n_gen) if N.gen.tsg_gen_file_nonascii(seed, f)]
    pick |= set(nonascii)
    rng = np.random.default_rng(seed + 11)
    rand_bytes = 0
    for f in rng.permutation(n_gen):
        if rand_bytes >= random_gb * 1e9:
            break
        if int(f) not in pick:
            pick.add(int(f))
            rand_bytes += int(sizes[f])
    pick = sorted(f for f in pick if f < n_gen)
    paths = c["d_paths"].cpu().numpy()
    items = [(f, int(sizes[f]), bytes(paths[f * 31:(f + 1) * 31]).decode()) for f in pick]
    items.sort(key=lambda x: -x[1])  # largest first: the pool ends together
    total = sum(x[1] for x in items)
    print(f"oracle parity: {len(items)} files, {total / 1e9:.2f} GB on {workers} processes", file=sys.stderr,
          flush=True)
    bad = []
    n_find = 0
    done = 0
    t_note = t0
    # spawned, not forked: the workers never hold this process's GPU handles
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers, initializer=_oracle_worker_init, initargs=(N.GEN_PATH, seed, density)) as pool:
        for k, (f, want) in enumerate(pool.imap_unordered(_oracle_worker, items, chunksize=1)):
            got = sorted(result_findings(N, res, f, rules))
            n_find += len(want)
            if got != want:
                bad.append(f)
            done += 1
            if done % 20000 == 0 or time.perf_counter() - t_note > 30:
                t_note = time.perf_counter()
                print(f"oracle parity: {done}/{len(items)} files, {len(bad)} mismatched, "
                      f"{time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)
    return dict(checker="oracle/secret_oracle.py (Python regex engine, independent of the engine's parser and VM)",
                files=len(items), bytes=total, plant_or_decoy_files=n_plant, gpu_finding_files=len(gpu_files),
                nonascii_files=len(nonascii), random_bytes=rand_bytes, findings=n_find,
                files_identical=len(items) - len(bad), mismatched=bad[:10], workers=workers,
                wall_seconds=round(time.perf_counter() - t0, 1))


def shared_layers_main(args, N, S, torch, dist, barrier, rank, world, device, red_dev):
    """configs[3] as one shared image: every rank derives the same layer list
    (shared_layer_set), trivy_amd.shard.partition assigns layers to ranks by
    bytes (LPT), each rank builds ITS layers as ustar tars in host memory, and
    a timed step is one trivy_amd.shard.scan_sharded call: the rank's layers
    walked on host threads ahead of one tsg_analyze_layer per layer, then the
    per-layer results (kept member indices + locations) gathered to every rank
    over the process group (all_gather_object) and returned in layer order --
    the reference's per-layer fan-out (pkg/fanal/artifact/image/image.go:201-240)
    with its merge.  Parity: --dump writes the merged result, which must not
    depend on the number of ranks (tests/test_bench_shared.py)."""
    from concurrent.futures import ThreadPoolExecutor

    from trivy_amd import shard

    n_layers = args.total_layers or args.layers * world
    layer_gb = shared_layer_set(args.seed, args.image_gb or args.gb * world, n_layers)
    plan = shard.partition([int(g * 1e9) for g in layer_gb], world)
    mine = plan[rank]
    sc = S.new_scanner(None, device=device)
    eng = S.get_engine(device)
    rs = sc._rs.handle
    t_tar = time.perf_counter()
    tars = {}
    content = {}
    for k in mine:
        ck = build_corpus(N, torch, args.seed + 7919 * k, layer_gb[k], args.density, device)
        host = ck["d_data"][: ck["packed"]].cpu().numpy()
        poff = ck["d_poff"].cpu().numpy().astype(np.int64)
        pbytes = ck["d_paths"][: int(poff[-1])].cpu().numpy()
        tars[k] = (ck["n_files"], build_layer_tar(host, ck["off"], ck["sizes"], pbytes, poff))
        content[k] = ck["total"]
        del ck, host
    torch.cuda.empty_cache()
    build_s = time.perf_counter() - t_tar
    pool = ThreadPoolExecutor(max_workers=4)

    def walk_one(layer):
        w = ctypes.c_void_p()
        N.check(N.lib.tsg_layer_tar_walk(ctypes.c_void_p(layer.ctypes.data), len(layer), None, 0, None, 0,
                                         ctypes.byref(w)))
        return w

    scan_ms = []

    def scan_fn(idxs):
        """This rank's layers, pipelined: walks run ahead on host threads, one
        analyze per layer; returns (kept member indices, locations) per layer."""
        futs = [pool.submit(walk_one, tars[k][1]) for k in idxs]
        out, ms = [], 0.0
        for k, f in zip(idxs, futs):
            nf, x = tars[k]
            w = f.result()
            kept = (ctypes.c_uint32 * (nf + 1))()
            nk = ctypes.c_size_t()
            r = ctypes.c_void_p()
            try:
                N.check(N.lib.tsg_analyze_layer(eng, rs, ctypes.c_void_p(x.ctypes.data), len(x), w, b"", kept,
                                                ctypes.byref(nk), ctypes.byref(r)))
            finally:
                N.lib.tsg_tar_walk_free(w)
            try:
                locs, tm = read_result(N, r)
            finally:
                N.lib.tsg_result_free(r)
            ms += tm[17] if len(tm) > 17 and tm[17] > 0 else tm[7]
            out.append((np.ctypeslib.as_array(kept)[: nk.value].copy(), locs))
        scan_ms.append(ms)
        return out

    sizes = [int(g * 1e9) for g in layer_gb]
    step = lambda: shard.scan_sharded(scan_fn, list(range(n_layers)), sizes=sizes)  # noqa: E731
    merged = None
    for _ in range(args.warmup):
        merged = step()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        merged = step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    mine_bytes = float(sum(content[k] for k in mine))
    if dist is not None:
        t = torch.tensor([dt], device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        tb = torch.tensor([mine_bytes], device=red_dev, dtype=torch.float64)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        total_all = float(tb.item())
    else:
        total_all = mine_bytes
    if rank == 0 and args.dump and merged is not None:
        arrs = {}
        for k, (kept, locs) in enumerate(merged):
            arrs[f"kept{k}"] = kept
            arrs[f"locs{k}"] = locs
        np.savez(args.dump, **arrs)
    if rank == 0:
        n_found = sum(len(locs) for _, locs in merged) if merged else 0
        out = {
            "metric": "secret-scan GB/s (whole node), builtin rules, 1/2/4/8 MI355X; % HBM peak",
            "value": round(total_all * args.steps / dt / 1e9, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak" if not args.image_gb else "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded SURVEY.md §8(d) text model, builtin-rule secrets planted at "
                    f"{args.density:g}/byte, one corpus seed per layer)",
            "config": {"workload": "configs[3]: ONE shared image of %d layers (%.3f GB) LPT-partitioned over the "
                                   "ranks by bytes (trivy_amd.shard.scan_sharded); per rank: native layer walks "
                                   "on host threads + one tsg_analyze_layer per layer; per-layer results gathered "
                                   "to every rank in the step; PCIe-inclusive" % (n_layers, total_all / 1e9),
                       "layers": n_layers, "layers_per_rank": [len(p) for p in plan],
                       "bytes_per_rank": [int(sum(sizes[k] for k in p)) for p in plan],
                       "dist_backend": args.dist_backend if world > 1 else None,
                       "layer_build_s": round(build_s, 1),
                       "parallelism": f"layer shards x{world} (LPT), all_gather of per-layer results"},
            "stages_ms": {"scan_kernels_rank0": round(float(np.mean(scan_ms[-args.steps:])), 3)},
            "counts": {"locs": int(n_found)},
            "roofline": None,
            "cpu_baseline": None,
            "parity": None,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=[0, 1, 2, 3, 4],
                    help="BASELINE.json configs index: 2 full ruleset (default), 0 analyzer batch from host "
                         "memory (PCIe-inclusive), 1 prefilter only, 3 layer tar per GPU (PCIe-inclusive), 4 stress rules")
    ap.add_argument("--gb", type=float, default=None, help="corpus GB per GPU (configs[2]: 50, configs[1]: 20)")
    ap.add_argument("--stress-rules", type=int, default=1000)
    ap.add_argument("--layers", type=int, default=4, help="configs[3]: layers per GPU")
    ap.add_argument("--density", type=float, default=1e-6)
    ap.add_argument("--seed", type=int, default=20261015 + 2)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-cores", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--full-parity", action="store_true",
                    help="after the timed steps, compare EVERY file's complete findings with the C++ restatement "
                         "(configs[2]; configs[4]: the unique C5 files + --full-parity-gb of text)")
    ap.add_argument("--full-parity-gb", type=float, default=0.0, help="--full-parity: limit to the first GB")
    ap.add_argument("--oracle-parity", action="store_true",
                    help="configs[2]: the Python oracle over every plant / decoy / finding / non-ASCII file "
                         "and --oracle-random-gb of random files (independent checker)")
    ap.add_argument("--oracle-random-gb", type=float, default=1.0)
    ap.add_argument("--staged", action="store_true",
                    help="configs[0] through the caller-filled page-locked staging (tsg_staging_add + "
                         "tsg_analyze_staged, as the tagged Go build's analyzer): the step copies every file into "
                         "its slot (16 threads) and runs the staged call")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N > 1 (nccl = RCCL; gloo for several ranks on one GPU in tests)")
    ap.add_argument("--shared", action="store_true",
                    help="configs[3] as ONE shared layer list: every rank sees the same image, layers are "
                         "LPT-partitioned by bytes (trivy_amd.shard), each rank builds and analyzes its layers, "
                         "and the per-layer results are gathered to every rank inside the timed step")
    ap.add_argument("--total-layers", type=int, default=0, help="--shared: layers in the image (default layers x N)")
    ap.add_argument("--image-gb", type=float, default=0.0,
                    help="--shared: bytes of the whole image (default --gb x N: fixed work per GPU)")
    ap.add_argument("--dump", default="", help="--shared: rank 0 writes the merged per-layer results (.npz)")
    args = ap.parse_args()
    if args.gb is None:
        args.gb = {0: 1.0, 1: 20.0, 3: 4.0, 4: 10.0}.get(args.config, 50.0)
    if args.shared and args.config != 3:
        ap.error("--shared is the configs[3] layer-set mode")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    # ranks beyond the visible GPUs share them (gloo tests: two ranks on one GPU);
    # device_count() does not initialise the GPU
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
    # reductions of the timing live on the GPU for RCCL, on the host for gloo
    red_dev = "cuda" if args.dist_backend == "nccl" else "cpu"

    def barrier():
        if dist is not None:
            dist.barrier()

    os.environ["TSG_DEVICE"] = str(device)
    from trivy_amd import _native as N
    import trivy_amd.secret as S

    if args.shared:
        return shared_layers_main(args, N, S, torch, dist, barrier, rank, world, device, red_dev)
    seed = args.seed + 1000 * rank
    c = build_corpus(N, torch, seed, args.gb, args.density, device)
    torch.cuda.synchronize()
    cfg = None
    stress_unique = []
    if args.config == 4:
        import tempfile

        from tests import stress_rules

        srules = stress_rules.make_rules(20261019, args.stress_rules)
        cfg_path = os.path.join(tempfile.mkdtemp(), "trivy-secret.yaml")
        stress_rules.write_config(cfg_path, srules)
        cfg = S.parse_config(cfg_path)
        # custom-rule instances (~1 per 4 lines), a 16 MiB
        # minified line and binary-ish files, appended to the HBM corpus as 2 %
        # of its bytes (~0.6 M findings: 20x the builtin plants' findings)
        stress_unique, stress_all = stress_material(stress_rules, srules, seed, int(c["total"] * 0.02))
        c = append_files(torch, c, stress_all, device)
    sc = S.new_scanner(cfg, device=device)
    eng = S.get_engine(device)
    rs = sc._rs.handle
    c["rs_handle"] = rs
    c["poff_host"] = c["d_poff"].cpu().numpy().astype(np.int64)
    st = [ctypes.c_uint32() for _ in range(4)]
    fast = ctypes.c_int()
    N.check(N.lib.tsg_ruleset_stats(rs, *[ctypes.byref(x) for x in st], ctypes.byref(fast)))
    # k_scan_fast when the automaton fits its LDS image, else k_scan_lines (the
    # configs[4] automaton: dense + sparse rows in LDS); both are bracketed by
    # the engine's HIP events (timings[17])
    scan_kernel = "k_scan_fast" if fast.value else "k_scan_lines"
    gate_words = (len(sc.rules) + 31) // 32
    gates = (ctypes.c_uint32 * (c["n_files"] * gate_words))() if args.config == 1 else None

    host_files = None
    if args.config == 0:
        # configs[0]: the files of a 1 GB source tree already read into host
        # memory (one packed host copy; every file handed over by pointer),
        # through the batched SecretAnalyzer front end: pinned staging + H2D,
        # IsBinary, '\r' deletion, scan, findings on the host
        host = c["d_data"][: c["packed"]].cpu().numpy()
        poff = c["d_poff"].cpu().numpy().astype(np.uint64)
        pbytes = c["d_paths"][: int(poff[-1])].cpu().numpy().tobytes()
        host_files = (N.FileC * c["n_files"])()
        base = host.ctypes.data
        path_objs = [pbytes[int(poff[i]):int(poff[i + 1])] for i in range(c["n_files"])]
        for i in range(c["n_files"]):
            host_files[i].data = ctypes.c_void_p(base + int(c["off"][i]))
            host_files[i].len = int(c["sizes"][i])
            host_files[i].path = path_objs[i]
        c["host_keep"] = (host, path_objs)
        if args.staged:
            st = ctypes.c_void_p()
            N.check(N.lib.tsg_staging_create(int(c["packed"]) + c["n_files"] + (1 << 20), ctypes.byref(st)))
            blib = cpu_lib()
            blib.tsgb_stage_files.restype = ctypes.c_size_t
            blib.tsgb_stage_files.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            s_off = np.ascontiguousarray(c["off"][: c["n_files"]], dtype=np.uint64)
            s_len = np.ascontiguousarray(c["sizes"][: c["n_files"]], dtype=np.uint64)
            s_paths = (ctypes.c_char_p * c["n_files"])(*path_objs)
            add_fn = ctypes.cast(N.lib.tsg_staging_add, ctypes.c_void_p)
            threads = min(16, cpu_quota())

            def staged_step():
                N.lib.tsg_staging_reset(st)
                k = blib.tsgb_stage_files(st, add_fn, ctypes.c_void_p(base), s_off.ctypes.data, s_len.ctypes.data,
                                          s_paths, c["n_files"], threads)
                if k != c["n_files"]:
                    raise RuntimeError(f"staging took {k} of {c['n_files']} files")
                r = ctypes.c_void_p()
                N.check(N.lib.tsg_analyze_staged(eng, rs, st, ctypes.byref(r)))
                return r
            c["staged_step"] = staged_step
            c["staged_keep"] = (st, s_off, s_len, s_paths, blib)

    layers = None
    if args.config == 3:
        # configs[3]: this rank's shard of the layer set, as `--layers` ustar
        # layers in host memory (the corpus files split in order); a step
        # walks them natively on host threads, pipelined ahead of the engine,
        # and analyzes each layer in one call (tsg_layer_tar_walk +
        # tsg_analyze_layer), as trivy_amd.walker.analyze_layers does
        from concurrent.futures import ThreadPoolExecutor

        host = c["d_data"][: c["packed"]].cpu().numpy()
        poff = c["d_poff"].cpu().numpy().astype(np.int64)
        pbytes = c["d_paths"][: int(poff[-1])].cpu().numpy()
        t_tar = time.perf_counter()
        cuts = np.linspace(0, c["n_files"], args.layers + 1).astype(np.int64)
        layers = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            layers.append((int(a), build_layer_tar(host, c["off"][a:b + 1], c["sizes"][a:b], pbytes,
                                                   poff[a:b + 1])))
        del host
        c["layer_build_s"] = time.perf_counter() - t_tar
        c["layer_bytes"] = sum(len(x) for _, x in layers)
        pool = ThreadPoolExecutor(max_workers=min(4, args.layers))
        c["kept"] = [(ctypes.c_uint32 * (int(b - a) + 1))() for a, b in zip(cuts[:-1], cuts[1:])]
        c["n_kept"] = [ctypes.c_size_t() for _ in layers]

    def walk_one(layer):
        w = ctypes.c_void_p()
        N.check(N.lib.tsg_layer_tar_walk(ctypes.c_void_p(layer.ctypes.data), len(layer), None, 0, None, 0,
                                         ctypes.byref(w)))
        return w

    trace_c3 = os.environ.get("TSG_C3_TRACE") is not None  # per-layer phase times on stderr

    if args.config == 3:  # layer k on engine k % 2 (trivy_amd.walker.analyze_layers' pipelining)
        from trivy_amd.secret import get_engines
        layer_engs = get_engines(device, 2)
        apool = ThreadPoolExecutor(max_workers=len(layer_engs))

    def layer_step():
        # one tsg_result per layer; the step returns the last (timings) and
        # frees the others after reading their counts
        t0 = time.perf_counter()
        futs = [pool.submit(walk_one, x) for _, x in layers]

        def one(k, x, f):
            w = f.result()
            t1 = time.perf_counter()
            r = ctypes.c_void_p()
            try:
                N.check(N.lib.tsg_analyze_layer(layer_engs[k % len(layer_engs)], rs, ctypes.c_void_p(x.ctypes.data),
                                                len(x), w, b"", c["kept"][k], ctypes.byref(c["n_kept"][k]),
                                                ctypes.byref(r)))
            finally:
                N.lib.tsg_tar_walk_free(w)
            if trace_c3:
                print(f"c3 layer {k}: walk ready {1e3 * (t1 - t0):.1f} ms, analyze {1e3 * (time.perf_counter() - t1):.1f} ms",
                      file=sys.stderr)
            return r
        afuts = [apool.submit(one, k, x, f) for k, ((_, x), f) in enumerate(zip(layers, futs))]
        return [a.result() for a in afuts]

    def one_step():
        if args.config == 3:
            for r in c.pop("layer_results", []):  # the previous step's non-last layers
                N.lib.tsg_result_free(r)
            rs_ = layer_step()
            c["layer_results"] = rs_[:-1]
            c["layer_scan_ms"] = sum(result_timings(N, r)[17] for r in rs_)
            return rs_[-1]
        if args.config == 0 and args.staged:
            return c["staged_step"]()
        if args.config == 0:
            r = ctypes.c_void_p()
            N.check(N.lib.tsg_analyze(eng, rs, host_files, c["n_files"], ctypes.byref(r)))
            return r
        if args.config == 1:
            N.check(N.lib.tsg_gate_device(eng, rs, ctypes.c_void_p(c["d_data"].data_ptr()),
                                          ctypes.c_void_p(c["d_off"].data_ptr()), c["n_files"], gates, gate_words))
            return None
        return scan_device(N, eng, rs, c)

    if args.config == 3:  # every member is required: result file i of layer k == corpus file cuts[k] + i
        for k, r in enumerate(layer_step()):
            N.lib.tsg_result_free(r)
            nk = c["n_kept"][k].value
            assert nk == int(cuts[k + 1] - cuts[k]) and all(c["kept"][k][i] == i for i in range(0, nk, 997))
    # warm-up steps keep the previous result alive as the timed loop does, so
    # the engine's pinned pool already holds the two result blocks it cycles
    prev = None
    for _ in range(args.warmup):
        r = one_step()
        if prev is not None:
            N.lib.tsg_result_free(prev)
        prev = r
    if prev is not None:
        N.lib.tsg_result_free(prev)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stage = None
    scan_ms = []
    # a step = one tsg_scan_device call: every kernel, the D2H of all
    # locations and the host line fix-up; results stay in the tsg_result
    # (host memory) and are read into numpy once, after the timed region
    locs, res, last = None, None, None
    for i in range(args.steps):
        res = one_step()
        if res is None:  # prefilter only: timings of the engine's last call
            tm = gate_timings(N, eng)
        else:
            tm = result_timings(N, res)
            if last is not None:
                N.lib.tsg_result_free(last)
            last = res
        scan_ms.append(c["layer_scan_ms"] if args.config == 3 else
                       tm[17] if len(tm) > 17 and tm[17] > 0 else tm[7])
        stage = tm
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        tb = torch.tensor([float(c["total"])], device=red_dev, dtype=torch.float64)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        total_all = float(tb.item())
    else:
        total_all = float(c["total"])

    if last is not None and args.config == 3:  # merge the layers' locations into corpus file numbering
        parts = []
        for k, r in enumerate(c.pop("layer_results") + [last]):
            lk, _ = read_result(N, r)
            lk = lk.copy()
            lk["file"] += np.uint32(cuts[k])
            parts.append(lk)
            N.lib.tsg_result_free(r)
        locs = np.concatenate(parts)
    elif last is not None:
        locs, _ = read_result(N, last)
    ms_per_step = dt / args.steps * 1e3
    value = total_all * args.steps / dt / 1e9
    scan_kernel_ms = float(np.mean(scan_ms))
    traffic = traffic_bytes(c["total"], scan_kernel) if args.config in (2, 4) else (None, None)
    achieved = c["total"] / (scan_kernel_ms / 1e3) / 1e9
    parity = None
    if rank == 0 and not args.no_parity:
        if args.config == 1:
            parity = gate_checks(N, c, sc.rules, gates, gate_words, seed, args.density)
        else:
            parity = parity_checks(N, S, c, locs, sc.rules, seed, args.density,
                                   n_sample=300 if args.config == 2 else 24, oracle_cfg=cfg_path if cfg else None,
                                   res=last if args.config in (0, 2, 4) else None)
            if args.config == 4:
                parity.update(stress_checks(N, last, sc.rules, c, stress_unique, cfg_path))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.config in (0, 2):
        # every CPU this process may run on: the affinity set capped by the
        # cgroup quota (N = the cores used, stated)
        cores = args.cpu_cores or cpu_quota()
        cpu = cpu_baseline(N, c, last, args.cpu_seconds, cores)
    full = None
    if rank == 0 and args.full_parity and args.config in (2, 4) and last is not None:
        cores = args.cpu_cores or cpu_quota()
        if args.config == 2:
            lim = args.full_parity_gb
            nf = c["n_files"] if not lim else int(np.searchsorted(c["off"], int(lim * 1e9)))
            full = full_parity(N, c, last, cores, [(0, max(1, nf))],
                               "configs[2]: every file" if not lim else f"configs[2]: first {lim:g} GB")
        else:
            # the C5 material's unique files (stress-rule instances, binary-ish
            # files, the 1 MiB and 16 MiB minified lines) + the first
            # --full-parity-gb of the generated text
            f0 = c["first_stress"]
            nf = int(np.searchsorted(c["off"], int((args.full_parity_gb or 0.25) * 1e9)))
            full = full_parity(N, c, last, cores, [(f0, f0 + len(stress_unique)), (0, max(1, min(nf, f0)))],
                               f"configs[4]: the {len(stress_unique)} unique C5 files + the first "
                               f"{args.full_parity_gb or 0.25:g} GB of generated text")
    oracle_full = None
    if rank == 0 and args.oracle_parity and args.config == 2 and last is not None:
        oracle_full = oracle_parity(N, c, last, sc.rules, seed, args.density, args.oracle_random_gb,
                                    max(1, (args.cpu_cores or cpu_quota()) - 1))
    if last is not None and args.config != 3:
        N.lib.tsg_result_free(last)
    h2d = None
    if rank == 0 and args.config in (0, 3):
        # the PCIe floor of a PCIe-inclusive step: the step's input bytes as
        # one page-locked H2D at the rate measured here (1 GiB, 3 copies)
        n = int(min(c["total"], 1 << 30))
        hb = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        db = torch.empty(n, dtype=torch.uint8, device=device)
        db.copy_(hb, non_blocking=True)
        torch.cuda.synchronize()
        t_h = time.perf_counter()
        for _ in range(3):
            db.copy_(hb, non_blocking=True)
        torch.cuda.synchronize()
        rate = 3 * n / (time.perf_counter() - t_h)
        step_bytes = c["layer_bytes"] if args.config == 3 else c["total"]
        h2d = {"gbps": round(rate / 1e9, 2), "floor_ms": round(step_bytes / rate * 1e3, 3),
               "step_bytes": int(step_bytes)}
        del hb, db
    if rank == 0:
        out = {
            "metric": "secret-scan GB/s (whole node), builtin rules, 1/2/4/8 MI355X; % HBM peak",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded SURVEY.md §8(d) text model, builtin-rule secrets planted at "
                    f"{args.density:g}/byte, generated in HBM)",
            "config": {"workload": WORKLOADS[args.config] + (f" ({args.stress_rules} generated rules)"
                                                              if args.config == 4 else "")
                       + (" -- through the caller-filled staging (tsg_staging_add, 16-thread slot fill, "
                          "tsg_analyze_staged)" if args.config == 0 and args.staged else ""),
                       "gb_per_gpu": round(c["total"] / 1e9, 3), "files_per_gpu": c["n_files"],
                       "density": args.density, "parallelism": f"file shards x{world}, no collective",
                       **({"layer_tar_bytes": c["layer_bytes"], "layer_build_s": round(c["layer_build_s"], 1)}
                          if args.config == 3 else {})},
            "pct_hbm_peak": round(100.0 * value / (HBM_PEAK_GBPS * world), 2),
            **({"h2d_floor": h2d} if h2d else {}),
            "roofline": {"bound": "hbm", "kernel": scan_kernel, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic[0], "traffic_source": traffic[1],
                         "algorithmic_bytes_per_launch": c["total"],
                         "avg_launch_ms": round(scan_kernel_ms, 3)},
            "stages_ms": ({"prefilter_total": round(stage[0], 3), "scan_kernel": round(scan_kernel_ms, 3)}
                          if args.config == 1 else {k: round(v, 3) for k, v in zip(
                              ["path_gate", "scan_total", "expand", "sort_jobs", "verify", "exclude", "lines",
                               "scan_kernels"], stage)}),
            "counts": None if args.config == 1 else dict(zip(
                ["hits", "candidates", "jobs", "locs", "event_overflow", "events", "outputs", "verify_deferred"],
                [int(v) for v in stage[8:15] + stage[23:24]]),
                **({"arena_bytes": int(stage[24]), "match_bytes": int(stage[25])} if len(stage) > 25 else {})),
            "host_ms": {"call_wall": round(stage[15], 3), "post": round(stage[16], 3),
                        **({"pack": round(stage[18], 3), "h2d": round(stage[19], 3)}
                           if len(stage) > 19 and args.config in (0, 3) else {}),
                        **({"front": round(stage[20], 3), "pipeline": round(stage[21], 3),
                            "findings": round(stage[22], 3)} if len(stage) > 22 and args.config in (0, 3) else {})},
            "cpu_baseline": cpu,
            "parity": parity,
            **({"full_parity": full} if full is not None else {}),
            **({"oracle_parity": oracle_full} if oracle_full is not None else {}),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
